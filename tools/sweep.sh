#!/bin/bash
# Engine-knob sweep on the GPU box (run from the repo root): one short bench per
# setting, each under its own time limit; stops at the first failure.
# usage: tools/sweep.sh <tag> <config> "<knobs>" ["<knobs>" ...]
#   e.g. tools/sweep.sh s1 tb_uniform "" "scatter_per_cu=1" "scatter_per_cu=2"
set -o pipefail
TAG=${1:-s}; CFG=${2:-tb_uniform}; shift 2
mkdir -p gpurun_out
i=0
for knobs in "$@"; do
  targs=""
  for kv in $knobs; do targs="$targs --tune $kv"; done
  log=gpurun_out/sweep_${TAG}_${CFG}_$i.log
  timeout -k 10 200 python -u bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline $targs > $log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$knobs] rc=$rc"; tail -3 $log; exit $rc; fi
  tail -1 $log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$knobs]', '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.05})"
  i=$((i+1))
done
