# C4 direction-split walks: triangle parity (kernels, golden, fixture, distributed routes), then the C4
# line with split lists (default) and combined lists (CAPSMI_TRI_SPLIT=0) for A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_triangles.py tests/test_gpu_fused_golden.py tests/test_gpu_dist_route.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/split_on.log 2>&1 || exit $?
CAPSMI_TRI_H16=0 timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/split_h16off.log 2>&1 || exit $?
CAPSMI_TRI_SPLIT=0 timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/split_off.log 2>&1 || exit $?
