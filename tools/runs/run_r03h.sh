#!/bin/bash
# routed results read in place by the unpermute (mid over normal records only), auto hot threshold;
# scatter0 component ablations (timing only) and unpermute grid A/B on sw_zipf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_h.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/t_h.log | head -20; tail -20 gpurun_out/t_h.log; exit 1; }
tail -1 gpurun_out/t_h.log
for v in "base" "noRec --tune ablate=1" "seqRec --tune ablate=2" "noMatch --tune ablate=4" "noPos --tune ablate=8" "noBar --tune ablate=16" "un2 --tune unpermute_per_cu=2" "un4 --tune unpermute_per_cu=4"; do
  set -- $v; tag=$1; shift
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra --steps 5 "$@" > gpurun_out/b_h_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 gpurun_out/b_h_$tag.log; exit 1; }
  tail -1 gpurun_out/b_h_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], {k: round(v,2) for k,v in d['stage_ms'].items()})"
done
