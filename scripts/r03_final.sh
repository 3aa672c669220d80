# End-of-round check (usage via gpurun: bash scripts/r03_final.sh): GPU suite, smoke, default bench,
# then the C4 profile set (bench + kernel trace + FETCH/WRITE PMC passes, scripts/run_full.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_suite.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || exit $?
bash scripts/run_full.sh r03_c4 c4
