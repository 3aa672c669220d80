# bench (with CPU baseline) + rocprofv3 kernel trace + FETCH/WRITE PMC passes; usage: bash scripts/run_full.sh TAG [workload]
# (PMC_MODES=cold,count: the C3 count(*) kernels get counters in the same summary)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-full}
W=${2:-c3}
B="python3 bench.py --workload $W --steps 3 --warmup 1 --modes ${PMC_MODES:-cold} --no-cpu-baseline"
: > gpurun_out/${T}_status.txt
timeout -k 10 400 python3 bench.py --workload $W --steps 5 --warmup 2 ${BENCH_MODES:-} > gpurun_out/${T}_bench.log 2>&1 || exit $?
echo bench ok >> gpurun_out/${T}_status.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.log 2>&1 || exit $?
echo trace ok >> gpurun_out/${T}_status.txt
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d gpurun_out/${T}_pmc_fetch -o run -- $B > gpurun_out/${T}_pmc_fetch.log 2>&1 || exit $?
echo pmc fetch ok >> gpurun_out/${T}_status.txt
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d gpurun_out/${T}_pmc_write -o run -- $B > gpurun_out/${T}_pmc_write.log 2>&1 || exit $?
echo pmc write ok >> gpurun_out/${T}_status.txt
