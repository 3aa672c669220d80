# Round 4: the distributed and new single-GPU parity tests only (one pytest process).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-t}
shift
SEL="$*"
timeout -k 10 900 python -u -m pytest ${SEL:-tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py tests/test_gpu_triangles.py tests/test_gpu_varlen.py tests/test_gpu_routing.py tests/test_gpu_ingest.py tests/test_gpu_undirected.py tests/test_gpu_count_star.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
