# Round 5 per-rank diagnostics on one GPU: every rank's C3 shard of 8 (owner(source) vs owner(target)), and the
# routed C5 / C3 lines rehearsed on 8 gloo ranks sharing the GPU with GPU work serialised (busy ms per rank).
# usage (on the box): WLS="c5 c3" bash scripts/r05_diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-g}
for BY in ${BYS:-source target}; do
  timeout -k 10 300 python -u bench.py --shard-of 8 --rels-by $BY --steps 5 --warmup 1 \
    > gpurun_out/${T}_shard8_$BY.log 2>&1 || exit $?
done
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-8000000000}
for W in ${WLS:-c5}; do
  A="--workload $W --steps 3 --warmup 1 --no-cpu-baseline"
  [ "$W" = c3 ] && A="$A --modes cold,count --scale ${C3SCALE:-26}"
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 900 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node ${NR:-8} --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus ${NR:-8} \
    $A > gpurun_out/${T}_${W}_rehearse${NR:-8}.log 2>&1 || exit $?
done
