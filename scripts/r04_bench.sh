# Round 4 measurements: the undirected 2-hop bench at s = 26, then the routed lines rehearsed on NR (8)
# gloo ranks sharing the GPU with GPU work serialised (per-rank busy ms; scripts/r04_dist.sh notes).
# usage (on the box): WLS="c4 c5" bash scripts/r04_bench.sh TAG [und]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-b}
if [ "${2:-und}" = und ]; then
  timeout -k 10 600 python -u bench.py --modes cold,count,und_count,und_distinct --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_und_bench.log 2>&1 || exit $?
fi
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-4000000000} CAPSMI_POOL_KEEP_BYTES=${CAPSMI_POOL_KEEP_BYTES:-4000000000}
for W in ${WLS:-c4 c5}; do
  A="--workload $W --steps 3 --warmup 1"
  [ "$W" = c3 ] && A="$A --modes ${C3MODES:-cold} --scale ${C3SCALE:-26}"
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node ${NR:-8} --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus ${NR:-8} $A > gpurun_out/${T}_${W}_rehearse${NR:-8}.log 2>&1 || exit $?
done
