# Round 5: the C3 bench at N = 2 rehearsed on one GPU (gloo ranks sharing the device, GPU work serialised),
# checking the multi-rank path of bench.py after the SURVEY 8d timing change; both relationship modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
for by in target source; do
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 \
    --steps 3 --warmup 1 --no-cpu-baseline --rels-by $by > gpurun_out/reh2_$by.log 2>&1 || exit $?
done
