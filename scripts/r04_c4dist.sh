# C4 over the distributed route: the parity tests, the route at world size 1 over RCCL, and the 2- and
# 8-rank gloo rehearsals.  usage (on the box): bash scripts/r04_c4dist.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${1:-c4d}
bash scripts/r04_tests.sh ${T} tests/test_gpu_dist_route.py tests/test_gpu_dist_golden.py tests/test_gpu_triangles.py || exit $?
CAPSMI_DIST_BACKEND=nccl RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29500 + RANDOM % 1000)) timeout -k 10 300 python -u bench.py --workload c4 --dist1 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_dist1.log 2>&1 || exit $?
NR=2 WLS="c4" bash scripts/r04_bench.sh ${T}2 none || exit $?
NR=8 WLS="c4" bash scripts/r04_bench.sh ${T}8 none
