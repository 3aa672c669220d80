# caching allocator: full GPU tests, then C5 / C3 cold with the cache on and off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/cache_tests.log 2>&1 || exit $?
for r in 1 2; do
  for w in c5 c3; do
    for cap in 1 0; do
      if [ $cap = 1 ]; then export CAPSMI_CACHE_BYTES=1; else unset CAPSMI_CACHE_BYTES; fi
      timeout -k 10 120 python3 bench.py --steps 5 --warmup 2 --modes cold --no-cpu-baseline --workload $w > gpurun_out/cache_${w}_cap${cap}_$r.log 2>&1 || exit $?
    done
  done
done
