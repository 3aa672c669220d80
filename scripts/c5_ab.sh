# C5 filter A/B: tests, base vs new, then sublog sweep of the new library
set -o pipefail
cd "$GRAFT_REPO_ROOT"
NEW=${NEW:-ab/pack.so}
CAPSMI_LIB=$PWD/$NEW timeout -k 10 300 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "varlen or optional" > gpurun_out/c5_tests.log 2>&1 || exit $?
BENCH_ARGS="--workload c5" bash scripts/ab.sh c5 ab/base.so $NEW || exit $?
for sl in 0 1 3; do
  CAPSMI_VL_DEBUG=1 CAPSMI_VL_SUBLOG=$sl CAPSMI_LIB=$PWD/$NEW timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --modes cold --no-cpu-baseline --workload c5 > gpurun_out/c5_sl$sl.log 2>&1 || exit $?
done
