# C3 count(*): parity (routing tests, var-length users of the chunk walker), then the count mode bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_varlen.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cab_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --modes count --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cab_part.log 2>&1 || exit $?
