# Round 5: C4 v-mode threshold sweep (CAPSMI_TRI_VMODE_T: od(v) from which a center's in-edges walk its
# out-list as v-mode) over the split lists: the C4 line per value (step, build, triangles, fixture check).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in 256 128 512 1024 64 256; do
  CAPSMI_TRI_VMODE_T=$t timeout -k 10 300 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline \
    >> gpurun_out/vmt_$t.log 2>&1 || exit $?
done
