#!/bin/bash
# A/B build of librl_engine.so with extra -D flags into distributed-rate-limiter_amd/variants/<name>/ (run here, on CPU).
# usage: tools/build_variant.sh <name> "<extra hipcc flags>" [git-rev]   (A/B: a revision with the constant changed)
#   git-rev: build that revision's sources (e.g. HEAD, the A/B base) instead of the working tree
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
out=$root/distributed-rate-limiter_amd/variants/$1; mkdir -p $out
src=$root
if [ -n "$3" ]; then
  src=$(mktemp -d); git -C "$root" archive "$3" distributed-rate-limiter_amd/csrc include | tar -x -C $src
fi
cd $src/distributed-rate-limiter_amd
F="-O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -Wall -Wno-unused-result $2"
objs=""
for s in csrc/rl_partition.hip csrc/rl_hot.hip csrc/rl_misc.hip csrc/rl_solo.hip csrc/rl_rt_*.hip csrc/rl_engine.cpp csrc/rl_router.cpp; do
  o=$out/$(basename ${s%.*}).o
  objs="$objs $o"
  /opt/rocm/bin/hipcc $F -x hip -c $s -o $o &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $out/librl_engine.so $objs
rm -f $out/*.o
[ "$src" != "$root" ] && rm -rf $src
echo built $out/librl_engine.so
