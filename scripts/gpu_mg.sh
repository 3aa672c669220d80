set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_rehearsal.py tests/test_gpu_routing.py -x -v --timeout 300 --timeout-method thread > gpurun_out/mg_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u bench.py --shard-of 8 --steps 5 --warmup 2 > gpurun_out/mg_shard8.log 2>&1 || exit $?
