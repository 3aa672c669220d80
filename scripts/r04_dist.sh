# Round 4: the distributed routes (C3/C4/C5 over gloo ranks and RCCL at world 1) and the single-GPU
# parity tests of the kernels they reuse; then the routed C4/C5 bench lines rehearsed on NR (8) gloo ranks, GPU work serialised.
# usage (on the box): bash scripts/r04_dist.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-dist}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py tests/test_gpu_triangles.py tests/test_gpu_varlen.py tests/test_gpu_routing.py tests/test_gpu_ingest.py tests/test_gpu_undirected.py tests/test_gpu_count_star.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
# the undirected 2-hop at s = 26 through the route (count(*): the record partition with both arcs), beside
# the directed cold / count(*) lines
timeout -k 10 600 python -u bench.py --modes cold,count,und_count,und_distinct --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_und_bench.log 2>&1 || exit $?
# the routed lines rehearsed on NR (8) gloo ranks sharing the GPU, GPU work serialised (per-rank busy ms);
# a small block cache per rank (8 processes share the device)
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-8000000000}
for W in ${WLS:-c4 c5 c3}; do
  A="--workload $W --steps 3 --warmup 1"
  [ "$W" = c3 ] && A="$A --modes cold,count --scale ${C3SCALE:-26}"
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node ${NR:-8} --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus ${NR:-8} $A > gpurun_out/${T}_${W}_rehearse${NR:-8}.log 2>&1 || exit $?
done
