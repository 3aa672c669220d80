# Round 5: k_rec_part specialised for full node filters (CAPSMI_REC_FULL=0 keeps the general form): parity of
# the count(*) paths, then the directed and undirected count(*) lines per form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_count_star.py tests/test_gpu_undirected.py tests/test_gpu_fused_golden.py \
  tests/test_gpu_routing.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/recfull_tests.log 2>&1 || exit $?
for f in 1 0 1; do
  CAPSMI_REC_FULL=$f timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recfull_$f.log 2>&1 || exit $?
done
