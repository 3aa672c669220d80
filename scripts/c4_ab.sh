# C4 v-block sweep: triangle tests, then the bench at several MALL budgets
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "triangle" > gpurun_out/c4_tests.log 2>&1 || exit $?
for mb in ${MBS:-0 128 64 256 32}; do
  CAPSMI_TRI_VBLOCK_MB=$mb timeout -k 10 200 python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_mb$mb.log 2>&1 || exit $?
done
