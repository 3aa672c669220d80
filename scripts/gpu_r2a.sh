set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2a_gputest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r2a_gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2a_bench.log 2>&1
