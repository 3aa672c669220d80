set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
echo "start $(date)" > gpurun_out/r1_status.txt
timeout -k 10 420 python -m pytest tests/test_gpu_graph.py -x -q > gpurun_out/r1_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/r1_status.txt
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1; echo "smoke rc=$?" >> gpurun_out/r1_status.txt
