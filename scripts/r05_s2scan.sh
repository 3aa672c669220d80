# Round 5: pass 2 (k_scatter_s2) with the single-wave scan of its 128 source-slice counters: partition / C3
# parity, then a same-box A/B of the headline against HEAD's library (libcapsmi_head.so via CAPSMI_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_part.py tests/test_gpu_graph.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py tests/test_gpu_dist_route.py tests/test_gpu_undirected.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/s2scan_tests.log 2>&1 || exit $?
H=$GRAFT_REPO_ROOT/cypher-for-apache-spark_amd/capsmi/libcapsmi_head.so
for i in 1 2 3; do
  CAPSMI_LIB=$H timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes cold \
    >> gpurun_out/s2scan_head.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes cold \
    >> gpurun_out/s2scan_new.log 2>&1 || exit $?
done
