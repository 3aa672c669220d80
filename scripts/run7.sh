set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/r7_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/r7_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --modes cold,warm,stream --no-cpu-baseline > gpurun_out/r7_bench.log 2>&1 && echo bench ok >> gpurun_out/r7_status.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r7_trace -o run -- python3 bench.py --steps 5 --warmup 2 --modes cold --no-cpu-baseline > gpurun_out/r7_trace.log 2>&1 && echo trace ok >> gpurun_out/r7_status.txt
