# Round 6: the distributed GPU tests (2 gloo ranks, RCCL at world size 1) and a 2-rank bench rehearsal of the
# default C3 line with count(*) (BY_TARGET, the complement-shard count).  usage: bash scripts/r06_dist.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-dist}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py tests/test_gpu_dist_rehearsal.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
CAPSMI_DIST_BACKEND=gloo CAPSMI_POOL_KEEP_BYTES=0 CAPSMI_CACHE_BYTES=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --scale 20 --steps 3 --warmup 1 --modes cold,count --no-cpu-baseline > gpurun_out/${T}_bench2.log 2>&1 || exit $?
