# radix join + pruned execution: GPU parity suite, then C2 through the generic joins (bench line + kernel trace)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rj_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload c2 --c2-route joins --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/rj_c2joins.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_c2joins -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c2 --c2-route joins --steps 2 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/rj_prof.log 2>&1
