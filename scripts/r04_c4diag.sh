# C4: the single-GPU line, the distributed route at world size 1 over RCCL (--dist1) with its kernel trace,
# and the 8-rank rehearsal.  usage (on the box): bash scripts/r04_c5diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-c5d}
export CAPSMI_DIST_BACKEND=nccl RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_single.log 2>&1 || exit $?
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python -u bench.py --workload c4 --dist1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_dist1.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c4 --dist1 --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_trace.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
unset RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR CAPSMI_DIST_BACKEND

