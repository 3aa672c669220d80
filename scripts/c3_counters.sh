# one SQ counter pass (VALU / LDS / VMEM instructions, waits, bank conflicts, L2 hit/miss) over the C3 cold line
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum -T -f csv -d gpurun_out/c3_sq -o run -- python3 bench.py --modes cold --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c3_sq.log 2>&1
