#!/bin/bash
# A/B build of librl_engine.so with extra -D flags into distributed-rate-limiter_amd/variants/<name>/ (run here, on CPU).
# usage: tools/build_variant.sh <name> "-DRL_TILE_ITEMS=64 ..."
set -e
cd "$(dirname "$0")/../distributed-rate-limiter_amd"
out=variants/$1; mkdir -p $out
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-result $2"
objs=""
for src in csrc/rl_partition.hip csrc/rl_hot.hip csrc/rl_misc.hip csrc/rl_rt_*.hip csrc/rl_engine.cpp csrc/rl_router.cpp; do
  o=$out/$(basename ${src%.*}).o
  objs="$objs $o"
  /opt/rocm/bin/hipcc $F -x hip -c $src -o $o &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/librl_engine.so $objs
echo built $out/librl_engine.so
