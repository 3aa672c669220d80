# C3 count(*): routing / parity tests, then the C3 bench with the count modes and a kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_fused_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cnt_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --modes cold,count,count_atomic --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/cnt_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cnt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --modes count --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/cnt_prof.log 2>&1
