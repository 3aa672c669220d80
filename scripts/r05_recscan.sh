# Round 5: k_rec_part with one packed scan for the runs and the pieces: count(*) parity, then the count(*)
# and undirected count(*) lines twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_count_star.py tests/test_gpu_undirected.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py tests/test_gpu_dist_route.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/recscan_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recscan_bench.log 2>&1 || exit $?
done
