set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/plan_new.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --plan-in-step > gpurun_out/plan_old.log 2>&1 || exit $?
