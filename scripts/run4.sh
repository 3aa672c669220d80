set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -q -m gpu > gpurun_out/r4_tests.log 2>&1
rc=$?; echo "tests rc=$rc" > gpurun_out/r4_status.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $B --layout clustered > gpurun_out/r4_clustered.log 2>&1 && echo clustered ok >> gpurun_out/r4_status.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r4_trace -o run -- $B > gpurun_out/r4_trace.log 2>&1 && echo trace ok >> gpurun_out/r4_status.txt && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex "k_hop|k_bitmap" -d gpurun_out/r4_fetch -o run -- $B > gpurun_out/r4_fetch.log 2>&1 && echo fetch ok >> gpurun_out/r4_status.txt && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_hop|k_bitmap" -d gpurun_out/r4_write -o run -- $B > gpurun_out/r4_write.log 2>&1 && echo write ok >> gpurun_out/r4_status.txt && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv --kernel-include-regex "k_hop" -d gpurun_out/r4_tcc -o run -- $B > gpurun_out/r4_tcc.log 2>&1 && echo tcc ok >> gpurun_out/r4_status.txt
