# Round 5: the undirected count(*) partition specialised for full node filters -- parity of the count paths, then
# the C3u lines (the und_count line first, as its own head line, and und_distinct).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_count_star.py tests/test_gpu_undirected.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/undfull_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --modes und_count,und_distinct --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/undfull_count.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --modes und_distinct,und_count --steps 10 --warmup 2 --no-cpu-baseline \
  > gpurun_out/undfull_distinct.log 2>&1 || exit $?
