# C2: parity (expand / routing / golden / table ops), bench lines (direct + planner route), kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_routing.py tests/test_gpu_golden.py tests/test_gpu_table_ops.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c2_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c2_direct.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c2 --c2-route planner --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c2_planner.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --c2-route planner --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/c2_prof.log 2>&1
