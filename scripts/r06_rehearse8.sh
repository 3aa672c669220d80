# Round 6 (complement shards for count(*)): the default C3 bench at N = 8 rehearsed on one GPU (8 gloo ranks sharing the device, GPU
# work serialised by a lock), the driver's scaling configuration at s = 24 (eight ranks of s = 26 do not fit one card); then N = 4.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-4000000000}
for n in 8 4; do
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n \
    --steps 3 --warmup 1 --no-cpu-baseline --scale 24 > gpurun_out/r06_reh_c3_$n.log 2>&1 || exit $?
done
