# generic joins: parity tests, then C2 through the planner (fused routing off) per join strategy, kernel trace of auto
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_radix_join.py tests/test_gpu_table_ops.py tests/test_gpu_routing.py tests/test_gpu_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || exit $?
for j in ${JOINS:-auto hash radix}; do
  CAPSMI_JOIN=$j timeout -k 10 300 python -u bench.py --workload c2 --c2-route joins --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$j.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ab_auto -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --c2-route joins --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/ab_prof.log 2>&1
