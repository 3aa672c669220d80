# Round 6: HIP API + kernel trace of the 1/8-sized C5 shard's routed step (world size 1 over RCCL, s = 17).
# usage (on the box): bash scripts/r06_c5api.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000))
T=${1:-c5api}
timeout -k 10 300 python3 bench.py --workload c5 --dist1 --scale 17 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_plain.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -T -f csv -d gpurun_out/${T}_trace -o run -- python3 bench.py \
  --workload c5 --dist1 --scale 17 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_trace.log 2>&1 || exit $?
