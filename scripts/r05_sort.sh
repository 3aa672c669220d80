# Sort pass forms and C4 walks: the sort users' parity tests, then the C4 line with the per-pass sort
# (default), the onesweep sort (CAPSMI_SORT=onesweep) and the combined-list walks (CAPSMI_TRI_SPLIT=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sort.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sort_tests0.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_triangles.py tests/test_gpu_radix_join.py tests/test_gpu_table_ops.py tests/test_gpu_graph.py tests/test_gpu_fused_golden.py tests/test_gpu_dist_route.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/sort_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sort_on.log 2>&1 || exit $?
CAPSMI_SORT=onesweep timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sort_off.log 2>&1 || exit $?
CAPSMI_TRI_SPLIT=0 timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sort_nosplit.log 2>&1 || exit $?
