# bench.py (short, no CPU baseline) per variant build: bash tools/bench_ab.sh <config> name1 name2 ...
set -o pipefail
C=$1; shift
for v in "$@"; do
  lib=distributed-rate-limiter_amd/variants/$v/librl_engine.so; [ "$v" = base ] && lib=
  RL_ENGINE_LIB=$lib timeout -k 10 200 python -u bench.py --config $C --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bab_${C}_$v.log 2>&1 || exit 1
  tail -1 gpurun_out/bab_${C}_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.05})"
done
