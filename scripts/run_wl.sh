# C2 / C4 / C5 bench lines (+ kernel trace of each); usage: bash scripts/run_wl.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-wl}
: > gpurun_out/${T}_status.txt
for w in c2 c4 c5; do
  timeout -k 10 500 python3 bench.py --workload $w --steps 5 --warmup 1 > gpurun_out/${T}_${w}.log 2>&1 || exit $?
  echo "$w ok" >> gpurun_out/${T}_status.txt
done
for w in c2 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${T}_trace_${w} -o run -- python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_trace_${w}.log 2>&1 || exit $?
  echo "$w trace ok" >> gpurun_out/${T}_status.txt
done
