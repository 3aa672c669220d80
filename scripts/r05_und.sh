# Round 5: the undirected 2-hop count(DISTINCT c) over the 2-D cell layout (csrc/k_und_part.hip).
# usage (on the box): bash scripts/r05_und.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-u}
timeout -k 10 600 python -u -m pytest tests/test_gpu_undirected.py tests/test_gpu_dist_route.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --modes und_distinct,und_count,cold --steps 5 --warmup 1 --no-cpu-baseline \
  > gpurun_out/${T}_und_bench.log 2>&1 || exit $?
