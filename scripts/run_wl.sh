# profile the single-GPU workloads: bash scripts/run_wl.sh TAG [workloads]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
T=${1:-wl}
for w in ${2:-c2 c4 c5}; do
  bash scripts/run_full.sh ${T}_$w $w || exit $?
done
