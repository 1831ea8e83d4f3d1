#!/bin/bash
# GPU-box driver for one iteration: smoke, GPU parity tests, 1-GPU bench (+ extra configs).
# usage: bash run_gpu.sh <tag> [config ...]      (default configs: tb_uniform)
set -o pipefail
TAG=${1:-x}; shift
CONFIGS=${@:-tb_uniform}
mkdir -p gpurun_out
timeout -k 10 150 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed rc=$?"; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in $CONFIGS; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --cpu-sample 16777216 > gpurun_out/bench_${TAG}_$c.log 2>&1; brc=$?
  echo "bench $c rc=$brc"
  [ $brc -eq 0 ] || exit $brc
  tail -1 gpurun_out/bench_${TAG}_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['workload'][:40], '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k:v for k,v in d['stage_ms'].items() if v>0.05})"
done
