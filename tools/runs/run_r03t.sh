#!/bin/bash
# config-1 stage breakdown; tb_uniform hot path on/off (idle k_hot_chains launch A/B), interleaved
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/config1_probe.py > gpurun_out/c1_probe.log 2>&1 || { tail -5 gpurun_out/c1_probe.log; exit 1; }
cat gpurun_out/c1_probe.log | grep -v amdgpu.ids
for rep in 1 2; do
  for v in on off; do
    t=""; [ $v = off ] && t="--tune hot_threshold=0"
    timeout -k 10 200 python -u bench.py --config tb_uniform --steps 20 --warmup 3 --no-cpu-baseline --no-extra $t > gpurun_out/b_t_${v}_${rep}.log 2>&1 || { tail -5 gpurun_out/b_t_${v}_${rep}.log; exit 1; }
    tail -1 gpurun_out/b_t_${v}_${rep}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tb hot $v', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'])"
  done
done
echo done
