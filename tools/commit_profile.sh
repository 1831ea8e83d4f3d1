#!/bin/bash
# Copy a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>/ (the CSVs the
# summary is computed from, flattened, plus a per-kernel summary.txt) and fold it into
# profiles/pmc_summary.json under <config>, citing profiles/<tag> (pmc_json --tag).
# usage: tools/commit_profile.sh <tag> <config> [pmc_json args...]
set -eo pipefail
TAG=$1; CFG=$2; shift 2
SRC=gpurun_out/prof_$TAG
DST=profiles/$TAG
mkdir -p $DST
cp $SRC/trace/trace_kernel_stats.csv $DST/
for f in fetch write tcc sq atomic; do
  [ -f $SRC/$f/${f}_counter_collection.csv ] && cp $SRC/$f/${f}_counter_collection.csv $DST/
done
python3 tools/prof_summary.py $SRC > $DST/summary.txt || true
python3 tools/pmc_json.py $DST $CFG --tag $DST "$@"
