# Round 5: C5 launch trimming (one zero launch for the accumulators, misfit flag, owned-range flags in k_final,
# pooled timer events) and the routed C2 / C4 / C5 bench steps pre-planned per SURVEY 8d: parity, the C5
# line, the 1/8-sized shard's trace and the 8-rank serialised rehearsal (scripts/r05_c5.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-c5b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_rehearsal.py tests/test_gpu_fused_golden.py tests/test_gpu_sparse_ids.py \
  -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests2.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 3 > gpurun_out/${T}_bench.log 2>&1 || exit $?
bash scripts/r05_c5.sh $T || exit $?
