# Round 6: parity of the partition / var-length / count paths, then the 1/8-sized C5 shard step, the whole C5
# line and the C3 cold line.  usage (on the box): bash scripts/r06_c5check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-c5chk}
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_part.py tests/test_gpu_count_star.py tests/test_gpu_graph.py tests/test_gpu_dist_route.py tests/test_gpu_fused_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
(export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000));
 timeout -k 10 300 python3 bench.py --workload c5 --dist1 --scale 17 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c5small.log 2>&1) || exit $?
timeout -k 10 300 python3 bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c5.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --modes cold --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3.log 2>&1 || exit $?
