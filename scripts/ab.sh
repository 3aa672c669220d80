# A/B of one bench line under library switches: bash scripts/ab.sh TAG "bench args" VAR=a VAR=b,W=c ...
# (a variant may set several variables, comma-separated)
# e.g. bash scripts/ab.sh joins "--workload c2 --c2-route joins" CAPSMI_JOIN=auto CAPSMI_JOIN=hash CAPSMI_JOIN=radix
#      bash scripts/ab.sh count "--modes count" CAPSMI_COUNT=part CAPSMI_COUNT=atomic
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
T=$1; ARGS=$2; shift 2
for kv in "$@"; do
  env ${kv//,/ } timeout -k 10 300 python3 bench.py $ARGS --steps 5 --warmup 2 --no-cpu-baseline > "gpurun_out/ab_${T}_${kv//[=\/,]/_}.log" 2>&1 || exit $?
done
