# Round 6: kernel trace of the C3 cold line (one step's timeline).  usage: bash scripts/r06_c3trace.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c3trace}
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -T -f csv -d gpurun_out/${T} -o run -- python3 bench.py \
  --modes cold --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}.log 2>&1 || exit $?
