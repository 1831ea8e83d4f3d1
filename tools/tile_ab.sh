# A/B of variant builds (tools/build_variant.sh) on the bench workload; one process per variant.
# usage: bash tools/tile_ab.sh "<variants for ablate.py>" name1 name2 ...   ("base" = the in-tree build)
set -o pipefail
V=$1; shift
for v in "$@"; do
  lib=distributed-rate-limiter_amd/variants/$v/librl_engine.so; [ "$v" = base ] && lib=
  RL_ENGINE_LIB=$lib timeout -k 10 120 python -u tools/ablate.py --config ${CFG:-tb_uniform} --rounds 5 --variants "$V" > gpurun_out/tile_$v.log 2>&1 || exit 1
done
