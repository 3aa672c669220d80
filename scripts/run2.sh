set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 420 python -m pytest tests/test_gpu_graph.py -q > gpurun_out/r2_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/r2_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --scale 22 --steps 5 --warmup 2 --cpu-scale 16 > gpurun_out/r2_b22.log 2>&1 && echo "b22 ok" >> gpurun_out/r2_status.txt && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2_b26.log 2>&1 && echo "b26 ok" >> gpurun_out/r2_status.txt
