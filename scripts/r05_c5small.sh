# Round 5: where a 1/8-sized C5 shard's time goes -- the distributed route at world size 1 over RCCL on an R-MAT
# of scale 17 (2^22 relationships, the size of one rank's shard of C5 at 8 ranks), under a kernel trace (a
# single rank: the process group from the environment, no launcher).
# usage (on the box): bash scripts/r05_c5small.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000))
T=${1:-c5s}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${T}_trace -o run -- python3 bench.py \
  --workload c5 --dist1 --scale 17 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_trace.log 2>&1 || exit $?
