# Round-5 profile set (usage via gpurun: bash scripts/r05_profiles.sh PART): PART a = C3 (cold, count(*),
# warm and the undirected count(*) kernels in one PMC summary) and C5; PART b = C2 and C4.  Bench lines with
# CPU baselines, kernel traces, FETCH/WRITE PMC passes (scripts/run_full.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
case "${1:-a}" in
  a)
    PMC_MODES=cold,count,warm,und_count,und_distinct bash scripts/run_full.sh r05_c3 c3 || exit $?
    bash scripts/run_full.sh r05_c5 c5 || exit $?
    ;;
  b)
    bash scripts/run_full.sh r05_c2 c2 || exit $?
    bash scripts/run_full.sh r05_c4 c4 || exit $?
    ;;
esac
echo "part ${1:-a} ok" > gpurun_out/r05_${1:-a}_done.txt
