# Round-2 profile refresh after the sort / count(*) / C4 changes: C3 (cold + count(*) kernels in one
# PMC summary), C4, and the C3 count(*) lines (record partition, pair partition, atomics).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
PMC_MODES=cold,count bash scripts/run_full.sh r02_c3 c3 || exit $?
bash scripts/run_full.sh r02_c4 c4 || exit $?
timeout -k 10 300 python3 bench.py --modes count,count_atomic --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_c3count_bench.log 2>&1 || exit $?
CAPSMI_COUNT=pairs timeout -k 10 300 python3 bench.py --modes count --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_c3count_pairs_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r02_c3count_trace -o run -- python3 bench.py --modes count --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c3count_trace.log 2>&1 || exit $?
echo all ok > gpurun_out/r02_refresh_done.txt
