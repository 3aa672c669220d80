# Round 6: C3 per-rank shard of 8 on one GPU, by source vs by target, with rank 0's per-kernel times.
# usage (on the box, via gpurun): bash scripts/r06_shard.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-shard}
for by in source target; do
  timeout -k 10 300 python -u bench.py --shard-of 8 --rels-by $by --steps 10 --warmup 3 > gpurun_out/${T}_${by}.json 2> gpurun_out/${T}_${by}.err || exit $?
done
