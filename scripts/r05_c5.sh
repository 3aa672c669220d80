# Round 5: C5 per-rank work -- var-length parity (single, sharded emulation, distributed routes), the 1/8-sized
# shard's kernel trace, then the routed C5 line rehearsed on 8 gloo ranks (GPU work serialised).
# usage (on the box): bash scripts/r05_c5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-c5}
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_dist_route.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
bash scripts/r05_c5small.sh ${T}s || exit $?
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-8000000000}
CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 8 \
  --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_rehearse8.log 2>&1 || exit $?
