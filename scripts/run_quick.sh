# tests + C3 bench + C2/C4/C5 bench lines; usage: bash scripts/run_quick.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-q}
: > gpurun_out/${T}_status.txt
timeout -k 10 600 python -u -m pytest tests -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${T}_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --modes cold,warm --no-cpu-baseline > gpurun_out/${T}_bench.log 2>&1 || exit $?
echo "bench ok" >> gpurun_out/${T}_status.txt
for w in ${WL:-c2 c4 c5}; do
  timeout -k 10 500 python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${w}.log 2>&1 || exit $?
  echo "$w ok" >> gpurun_out/${T}_status.txt
done
