# tests + bench only; usage: bash scripts/run_quick.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-q}
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/${T}_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --modes cold,warm --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 && echo bench ok >> gpurun_out/${T}_status.txt
