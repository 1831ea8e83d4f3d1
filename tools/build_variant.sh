#!/bin/bash
# A/B build of librl_engine.so with extra -D flags into distributed-rate-limiter_amd/variants/<name>/ (run here, on CPU).
# usage: tools/build_variant.sh <name> "-DRL_TILE_ITEMS=64 ..."
set -e
cd "$(dirname "$0")/../distributed-rate-limiter_amd"
out=variants/$1; mkdir -p $out
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-result $2"
/opt/rocm/bin/hipcc $F -c csrc/rl_kernels.hip -o $out/k.o &
/opt/rocm/bin/hipcc $F -x hip -c csrc/rl_engine.cpp -o $out/e.o &
/opt/rocm/bin/hipcc $F -x hip -c csrc/rl_router.cpp -o $out/r.o
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/librl_engine.so $out/k.o $out/e.o $out/r.o
echo built $out/librl_engine.so
