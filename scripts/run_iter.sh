# quick iteration: partition/graph parity tests + C3 bench; usage: bash scripts/run_iter.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-it}
K=${2:-"part or graph"}
: > gpurun_out/${T}_status.txt
timeout -k 10 400 python -u -m pytest tests -v -m gpu -k "$K" --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${T}_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --modes ${MODES:-cold} --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/${T}_status.txt
