# GPU check: parity tests, smoke, default bench; then (optional) the full C3 profile set
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-chk}
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
if [ -n "$2" ]; then bash scripts/run_full.sh ${T}_full $2 || exit $?; fi
