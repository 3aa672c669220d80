# Round 5: the 6-byte pass-1 pool of the C3 layout (csrc/k_part.hip k_scatter_l6): parity tests of every route
# that builds the layout, then the default bench and the 8-byte pool (CAPSMI_P1=8) as A/B on the same box.
# usage (on the box): bash scripts/r05_p1.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_part.py tests/test_gpu_graph.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py tests/test_gpu_undirected.py tests/test_gpu_dist_route.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench6.log 2>&1 || exit $?
CAPSMI_P1=8 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_bench8.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --modes cold > gpurun_out/${T}_bench6b.log 2>&1 || exit $?
