# Round 6 profile set: C3 (the metric; cold + count kernels in one PMC summary), then C2, C4, C5 -- each bench
# with its CPU baseline, a kernel trace and the FETCH / WRITE PMC passes (scripts/run_full.sh).
# usage (on the box): bash scripts/r06_profiles.sh [c3|rest|all]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
case "${1:-all}" in
  c3) PMC_MODES=cold,count bash scripts/run_full.sh r06_c3 c3 || exit $? ;;
  rest)
    bash scripts/run_full.sh r06_c2 c2 || exit $?
    bash scripts/run_full.sh r06_c4 c4 || exit $?
    bash scripts/run_full.sh r06_c5 c5 || exit $?
    ;;
  all)
    PMC_MODES=cold,count bash scripts/run_full.sh r06_c3 c3 || exit $?
    bash scripts/run_full.sh r06_c2 c2 || exit $?
    bash scripts/run_full.sh r06_c4 c4 || exit $?
    bash scripts/run_full.sh r06_c5 c5 || exit $?
    ;;
esac
