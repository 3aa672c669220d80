# Round 5: C4 build load merging (k_swap_keys_sp: three lane loads per edge; k_split_count / k_split_write: 16-byte loads):
# triangle parity, then the C4 line twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_triangles.py tests/test_gpu_fused_golden.py tests/test_gpu_routing.py \
  tests/test_gpu_dist_route.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/swapkeys_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline >> gpurun_out/swapkeys_c4.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/swapkeys_tr -o run -- python3 bench.py --workload c4 \
  --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/swapkeys_tr.log 2>&1 || exit $?
