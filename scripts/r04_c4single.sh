# the single-GPU C4 line with the build's phase timers
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${1:-c4}_c4single.log 2>&1
