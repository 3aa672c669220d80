set -o pipefail
cd "$GRAFT_REPO_ROOT"
for e in ${EXPS:-0 1 4}; do
  CAPSMI_EXP=$e timeout -k 10 120 python3 bench.py --steps 3 --warmup 1 --modes cold --no-cpu-baseline > gpurun_out/exp_$e.log 2>&1 || exit $?
done
