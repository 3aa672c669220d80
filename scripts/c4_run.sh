# C4: triangle parity (kernels, routing, golden, fixture), the C4 line,
# then a kernel trace and FETCH/WRITE passes of the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_triangles.py tests/test_gpu_routing.py tests/test_gpu_fused_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c4_tests.log 2>&1 || exit $?
bash scripts/run_full.sh ${1:-c4new} c4 || exit $?
