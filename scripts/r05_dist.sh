# Round 5: the one-distribution routes (BY_SOURCE) and library-level collective chunking.
# usage (on the box): bash scripts/r05_dist.sh TAG [tests|bench|all]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-d}
W=${2:-all}
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1"
if [ "$W" = tests ] || [ "$W" = all ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
fi
if [ "$W" = bench ] || [ "$W" = all ]; then
  for BY in source target; do
    timeout -k 10 300 $R --master-port $((29500 + RANDOM % 1000)) bench.py --dist1 --rels-by $BY --modes cold,count \
      --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_c3_dist1_$BY.log 2>&1 || exit $?
  done
  # the C4 build's 2^28-word exchange and all-gather at world size 1, every RCCL call cut by libcapsmi
  timeout -k 10 400 $R --master-port $((29500 + RANDOM % 1000)) bench.py --workload c4 --dist1 --steps 2 --warmup 1 \
    --no-cpu-baseline > gpurun_out/${T}_c4_dist1.log 2>&1 || exit $?
fi
