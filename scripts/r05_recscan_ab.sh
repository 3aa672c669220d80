# Round 5: same-box A/B of the packed runs+pieces scan -- HEAD's library (libcapsmi_head.so, CAPSMI_LIB) against
# the working tree's, alternating, the count(*) and undirected count(*) lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
H=$GRAFT_REPO_ROOT/cypher-for-apache-spark_amd/capsmi/libcapsmi_head.so
for i in 1 2 3; do
  CAPSMI_LIB=$H timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recab_head.log 2>&1 || exit $?
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --modes count,und_count \
    >> gpurun_out/recab_new.log 2>&1 || exit $?
done
