# A/B timing of library variants in one box: bash scripts/ab.sh TAG lib1.so lib2.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=$1; shift
for r in 1 2; do
  for v in "$@"; do
    n=$(basename $v .so)
    CAPSMI_LIB=$PWD/$v timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --modes ${MODES:-cold} --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/${T}_${n}_$r.log 2>&1 || exit $?
  done
done
