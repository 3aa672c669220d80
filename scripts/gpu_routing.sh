set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_routing.py -x -v --timeout 200 --timeout-method thread > gpurun_out/routing.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/routing.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpuall.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/gpuall.log
exit $rc
