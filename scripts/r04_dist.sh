# Round 4: the distributed routes (C3/C4/C5 over gloo ranks and RCCL at world 1) and the single-GPU
# parity tests of the kernels they reuse; then the routed C4/C5 bench lines rehearsed on 2 gloo ranks.
# usage (on the box): bash scripts/r04_dist.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-dist}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_route.py tests/test_gpu_triangles.py tests/test_gpu_varlen.py tests/test_gpu_routing.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
