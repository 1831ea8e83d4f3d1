#!/bin/bash
# 32-bit time reductions in k_hot_summ: hot/config/parity GPU tests, kernel trace of sw_zipf
set -o pipefail
mkdir -p gpurun_out
true
true
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_j -o trace -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/prof_j.log 2>&1 || { tail -5 gpurun_out/prof_j.log; exit 1; }
f=$(find gpurun_out/prof_j -name "*kernel_stats.csv" | head -1)
grep -E "k_hot_summ|k_scatter_split|k_unpermute" $f | cut -c1-160
echo done
