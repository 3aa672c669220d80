set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $B --layout clustered > gpurun_out/r3_clustered.log 2>&1 && echo clustered ok > gpurun_out/r3_status.txt && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/r3_trace -o run -- $B > gpurun_out/r3_trace.log 2>&1 && echo trace ok >> gpurun_out/r3_status.txt && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv --kernel-include-regex "k_hop|k_bitmap|k_popcount" -d gpurun_out/r3_fetch -o run -- $B > gpurun_out/r3_fetch.log 2>&1 && echo fetch ok >> gpurun_out/r3_status.txt && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv --kernel-include-regex "k_hop|k_bitmap|k_popcount" -d gpurun_out/r3_write -o run -- $B > gpurun_out/r3_write.log 2>&1 && echo write ok >> gpurun_out/r3_status.txt && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv --kernel-include-regex "k_hop" -d gpurun_out/r3_tcc -o run -- $B > gpurun_out/r3_tcc.log 2>&1 && echo tcc ok >> gpurun_out/r3_status.txt
