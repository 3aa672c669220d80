# Round 6: alternate library builds on one box (CAPSMI_LIB) for one bench line, twice each (A B A B ...).
# usage: bash scripts/r06_libab.sh TAG "bench args" lib1.so lib2.so ...   (paths relative to the repo root)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=$1; ARGS=$2; shift 2
for rep in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    CAPSMI_LIB="$GRAFT_REPO_ROOT/$lib" timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline > "gpurun_out/${T}_${name}_${rep}.log" 2>&1 || exit $?
  done
done
