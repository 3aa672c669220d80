# Round 5, end: the whole GPU suite (parity tests in one process, smoke, the default bench line), then the
# C2 and C4 profile sets (bench with CPU baseline, kernel trace, FETCH / WRITE passes; scripts/run_full.sh).
# usage (on the box, via gpurun): bash scripts/r05_final.sh [suite|profiles|all]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
case "${1:-all}" in
  suite) bash scripts/gpu_suite.sh r05f || exit $? ;;
  profiles)
    bash scripts/run_full.sh r05_c2 c2 || exit $?
    bash scripts/run_full.sh r05_c4 c4 || exit $?
    ;;
  all)
    bash scripts/gpu_suite.sh r05f || exit $?
    bash scripts/run_full.sh r05_c2 c2 || exit $?
    bash scripts/run_full.sh r05_c4 c4 || exit $?
    ;;
esac
echo "final ${1:-all} ok" > gpurun_out/r05_final_done.txt
