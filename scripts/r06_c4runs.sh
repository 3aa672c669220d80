# Round 6: the fused run passes of the direct C4 build -- triangle / C4 parity tests, then the C4 line
# A/B against the previous library (scripts/r06_libab.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=${1:-r06or}
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_triangles.py tests/test_gpu_fused_golden.py tests/test_gpu_determinism.py tests/test_gpu_dist_golden.py \
  > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -3 gpurun_out/${T}_tests.log
bash scripts/r06_libab.sh ${T} "--workload c4 --steps 5 --warmup 2" ab_libs/base.so ab_libs/orruns.so
for f in gpurun_out/${T}_*_?.log; do echo "$f"; grep -o '"ms_per_step": [0-9.]*' $f; grep -o '"tri_[a-z_]*": [0-9.]*' $f | tr '\n' ' '; grep -o '"check_vs_fixture": "[a-z]*"' $f; done
