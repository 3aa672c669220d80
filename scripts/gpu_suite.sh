# The GPU check of a round: parity tests (one pytest process), smoke, the default bench.
# usage (on the box, via gpurun): bash scripts/gpu_suite.sh TAG [tests-selector]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-suite}
timeout -k 10 900 python -u -m pytest ${2:-tests} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
