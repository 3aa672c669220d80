# Round 5: C4 work shares of 8 ranks timed one by one on one GPU (bench.py --tri-parts 8), plus the 6-byte
# pool test.  usage (on the box): bash scripts/r05_c4parts.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-c4p}
timeout -k 10 300 python -u -m pytest tests/test_gpu_part.py -m gpu -x -v -k six_byte --timeout 200 \
  --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --tri-parts 8 \
  > gpurun_out/${T}_c4parts.log 2>&1 || exit $?
