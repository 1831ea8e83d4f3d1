#!/bin/bash
# round 5: walk table init per listed region (the gate checked once per region and 4096-entry
# part instead of per entry): walk / hot parity, kernel trace of sw_zipf and mixed_tenants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_walk.py tests/test_gpu_hot.py -x -q --timeout 240 --timeout-method thread > gpurun_out/t_r05ae.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch|assert" gpurun_out/t_r05ae.log | head -20; tail -30 gpurun_out/t_r05ae.log; exit 1; }
tail -1 gpurun_out/t_r05ae.log
for cfg in sw_zipf mixed_tenants; do
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05ae_$cfg -o trace --output-format csv -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_r05ae_$cfg.log 2>&1 || { echo "trace $cfg failed"; tail -5 gpurun_out/prof_r05ae_$cfg.log; exit 1; }
f=$(find gpurun_out/prof_r05ae_$cfg -name "*kernel_stats.csv" | head -1)
grep -E "walk_init|hot_summ" $f | cut -c1-160
done
echo done
