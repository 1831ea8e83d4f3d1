#!/bin/bash
# same-box A/B: region occupancy 5 waves/SIMD, scatter prefetch depth 4, unpermute workgroups per CU
set -o pipefail
mkdir -p gpurun_out
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  RL_ENGINE_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline "$@" > gpurun_out/b_q_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_q_$tag.log; return 1; }
  tail -1 gpurun_out/b_q_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.1})"
}
AB=distributed-rate-limiter_amd/ab
for rep in 1 2; do
  run base_$rep "" || exit 1
  run rw5_$rep $AB/librl_engine_rw5.so || exit 1
  run sd4_$rep $AB/librl_engine_sd4.so || exit 1
  run un2_$rep "" --tune unpermute_per_cu=2 || exit 1
  run un4_$rep "" --tune unpermute_per_cu=4 || exit 1
  run up8_$rep "" --tune upsweep_per_cu=8 || exit 1
done
