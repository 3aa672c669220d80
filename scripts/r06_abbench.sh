# Round 6: the previous bench.py (every kernel timer inside the timed steps) against the current one (the dominant
# launch timed alone) on one box: C3 cold, C5, C2, the 1/8-sized C5 shard.  usage: bash scripts/r06_abbench.sh TAG
# bench_prev.py: `git show 6475bc3:bench.py > bench_prev.py` (not committed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=$1
for rep in 1 2; do
 for b in bench_prev bench; do
  timeout -k 10 300 python3 $b.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c3_${b}_${rep}.log 2>&1 || exit 1
  timeout -k 10 300 python3 $b.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c5_${b}_${rep}.log 2>&1 || exit 1
  timeout -k 10 300 python3 $b.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c2_${b}_${rep}.log 2>&1 || exit 1
  (export RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000)); timeout -k 10 300 python3 $b.py --workload c5 --dist1 --scale 17 --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/${T}_c5s_${b}_${rep}.log 2>&1) || exit 1
 done
done
