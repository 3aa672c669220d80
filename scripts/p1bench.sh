# build the pass-1 microbenchmark (after `make -C cypher-for-apache-spark_amd`); run ./scripts/p1bench on the GPU box
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-function -munsafe-fp-atomics \
  p1bench.hip -o p1bench -L../cypher-for-apache-spark_amd/capsmi -lcapsmi -Wl,-rpath,'$ORIGIN/../cypher-for-apache-spark_amd/capsmi'
