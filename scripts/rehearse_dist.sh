# Multi-rank rehearsal of the distributed bench lines on a one-GPU box: gloo ranks sharing the
# device (RCCL refuses two ranks per GPU); checks the sharded answers against the whole table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for n in ${NS:-2 4}; do
  for wl in ${WLS:-c3 c5 c2}; do
    CAPSMI_DIST_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --workload $wl --steps 2 --warmup 1 \
      --no-cpu-baseline > gpurun_out/rehearse_${wl}_n$n.log 2>&1 || exit $?
    grep -q '"check_vs_[a-z]*": "ok"' gpurun_out/rehearse_${wl}_n$n.log || exit 3
  done
done
