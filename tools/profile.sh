#!/bin/bash
# Profile the bench workload with rocprofv3 on the GPU box (run from the repo root):
#   kernel trace + stats, then one PMC pass per counter group (never combined with
#   tracing domains; each pass bounded by its own timeout).
# usage: tools/profile.sh <tag> [bench args...]     (tag e.g. r06_sw_zipf)
# Then, back in the build container: tools/commit_profile.sh <tag> <config> copies the CSVs
# to profiles/<tag>/ and folds them into profiles/pmc_summary.json with --tag profiles/<tag>
# (the directory bench.py's roofline.traffic_source cites).
set -o pipefail
TAG=${1:-r01}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 -s KILL 240 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run trace --kernel-trace --stats || exit 1
run fetch --pmc FETCH_SIZE || exit 1
run write --pmc WRITE_SIZE || exit 1
run tcc --pmc TCC_HIT_sum TCC_MISS_sum || exit 1
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY || exit 1
run atomic --pmc TCC_EA0_ATOMIC_sum || exit 1
echo done
