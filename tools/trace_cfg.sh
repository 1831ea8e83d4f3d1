#!/bin/bash
# rocprofv3 kernel trace (+stats) of one bench config on the GPU box.
# usage: bash tools/trace_cfg.sh <tag> <config> [bench args]
set -o pipefail
TAG=$1; CFG=$2; shift 2
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof_${TAG}_$CFG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 bench.py --config $CFG $ARGS > $OUT/trace.log 2>&1
echo "trace rc=$?"
