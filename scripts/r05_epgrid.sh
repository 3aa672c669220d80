# Round 5: C2 k_expand_pairs grid sweep (CAPSMI_EP_GRID workgroups per CU), the C2 line per value.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for g in 4 2 8 16 4; do
  CAPSMI_EP_GRID=$g timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline \
    >> gpurun_out/epgrid_$g.log 2>&1 || exit $?
done
