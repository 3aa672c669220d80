# Round-2 profile set: bench + kernel trace + FETCH/WRITE PMC passes for C3/C2/C4/C5, the C2 line through
# the generic joins, C3 count(*) (partitioned vs atomic), and L2 hit/miss counters of the C2 expand.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for w in c3 c2 c4 c5; do
  bash scripts/run_full.sh r02_$w $w || exit $?
done
timeout -k 10 300 python3 bench.py --workload c2 --c2-route joins --steps 5 --warmup 2 > gpurun_out/r02_c2joins_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r02_c2joins_trace -o run -- python3 bench.py --workload c2 --c2-route joins --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c2joins_trace.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --modes count,count_atomic --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_c3count_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r02_c3count_trace -o run -- python3 bench.py --modes count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c3count_trace.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv -d gpurun_out/r02_c2_pmc_l2 -o run -- python3 bench.py --workload c2 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c2_pmc_l2.log 2>&1 || exit $?
echo all ok > gpurun_out/r02_done.txt
