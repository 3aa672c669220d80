# Round 5: k_rec_part without the barrier between the held-record writes and the bookkeeping: count(*) parity,
# then a same-box A/B against HEAD's library (libcapsmi_head.so via CAPSMI_LIB), alternating.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_count_star.py tests/test_gpu_undirected.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py tests/test_gpu_dist_route.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/recbar_tests.log 2>&1 || exit $?
H=$GRAFT_REPO_ROOT/cypher-for-apache-spark_amd/capsmi/libcapsmi_head.so
for i in 1 2 3; do
  CAPSMI_LIB=$H timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recbar_head.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recbar_new.log 2>&1 || exit $?
done
