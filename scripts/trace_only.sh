# kernel traces of several workloads (cold): bash scripts/trace_only.sh TAG wl...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=$1; shift
for w in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${T}_${w} -o run -- python3 bench.py --workload $w --steps 3 --warmup 1 --modes cold --no-cpu-baseline > gpurun_out/${T}_${w}.log 2>&1 || exit $?
done
