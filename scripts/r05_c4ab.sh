# C4 A/B lines: the triangle parity tests (kernels, golden, distributed routes), the default line, then each
# CAPSMI_* setting given as an argument (e.g. CAPSMI_TRI_UBLOCK=1024; several in one quoted argument)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_triangles.py tests/test_gpu_fused_golden.py tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_default.log 2>&1 || exit $?
i=0
for kv in "$@"; do
  i=$((i + 1))
  env $kv timeout -k 10 300 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1 || exit $?
done
