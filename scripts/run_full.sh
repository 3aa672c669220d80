set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-full}
B="python3 bench.py --steps 3 --warmup 1 --modes cold --no-cpu-baseline"
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/${T}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/${T}_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 --modes cold,warm,stream > gpurun_out/${T}_bench.log 2>&1 && echo bench ok >> gpurun_out/${T}_status.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.log 2>&1 && echo trace ok >> gpurun_out/${T}_status.txt && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d gpurun_out/${T}_pmc_fetch -o run -- $B > gpurun_out/${T}_pmc_fetch.log 2>&1 && echo pmc fetch ok >> gpurun_out/${T}_status.txt && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d gpurun_out/${T}_pmc_write -o run -- $B > gpurun_out/${T}_pmc_write.log 2>&1 && echo pmc write ok >> gpurun_out/${T}_status.txt
