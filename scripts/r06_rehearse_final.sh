# Round 6, final tree: the default C3 bench and the C4 / C5 routed lines rehearsed at N = 2 and 4 (gloo ranks sharing the
# one GPU, GPU work serialised by a lock), s = 24 for C3 (C4 s = 20, C5 s = 18).  usage: bash scripts/r06_rehearse_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-rehf}
LOCK=$(mktemp /tmp/capsmi_serial.XXXXXX)
export CAPSMI_CACHE_BYTES=${CAPSMI_CACHE_BYTES:-4000000000}
run() {  # n, log, bench args...
  local n=$1 log=$2; shift 2
  CAPSMI_DIST_BACKEND=gloo CAPSMI_SERIAL_LOCK=$LOCK timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $n "$@" \
    > gpurun_out/${T}_$log.log 2>&1
}
run 2 c3_2 --steps 3 --warmup 1 --no-cpu-baseline --scale 24 || exit $?
run 4 c3_4 --steps 3 --warmup 1 --no-cpu-baseline --scale 24 --modes cold,count || exit $?
run 2 c4_2 --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --scale 20 || exit $?
run 2 c5_2 --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --scale 18 || exit $?
