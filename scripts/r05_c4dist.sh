# Round 5: C4 at 8 ranks rehearsed on one GPU (gloo, ranks sharing the device, GPU work serialised by
# CAPSMI_SERIAL_LOCK so each rank's phases are timed alone; the answer checked against the s = 24 fixture),
# and the 8 work shares of one single-GPU trigraph timed one by one.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --tri-parts 8 \
  > gpurun_out/c4d_parts.log 2>&1 || exit $?
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-8000000000}
CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 900 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 8 \
  --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4d_rehearse8.log 2>&1 || exit $?
