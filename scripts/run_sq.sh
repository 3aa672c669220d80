# SQ counter pass on the partition / hop kernels; usage: bash scripts/run_sq.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-sq}
: > gpurun_out/${T}_status.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --kernel-include-regex "k_scatter|k_hop" -T -f csv -d gpurun_out/${T}_pmc -o run -- python3 bench.py --steps 1 --warmup 0 --modes cold --no-cpu-baseline > gpurun_out/${T}_pmc.log 2>&1 && echo pmc ok >> gpurun_out/${T}_status.txt
