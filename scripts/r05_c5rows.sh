# Round 5: var-length rows written before their count is read (flags_to_rows): parity, then the 1/8-sized
# shard's trace (scripts/r05_c5small.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_dist_route.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py tests/test_gpu_sparse_ids.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/c5rows_tests.log 2>&1 || exit $?
bash scripts/r05_c5small.sh c5rows || exit $?
