# C3 at s = 26: the single-GPU route vs the distributed route at world size 1 over RCCL (bench.py
# --dist1: every exchange of the N > 1 path, trivially sized), plus a kernel trace of the latter.
# usage (on the box): bash scripts/r04_dist1.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-d1}
export CAPSMI_DIST_BACKEND=nccl RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1
timeout -k 10 300 python -u bench.py --modes cold,count --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_single.log 2>&1 || exit $?
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python -u bench.py --dist1 --modes cold,count --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_dist1.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof" -o dist1 -- python3 "$GRAFT_REPO_ROOT/bench.py" --dist1 --modes cold --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/${T}_prof.log" 2>&1
