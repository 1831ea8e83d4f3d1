#!/bin/bash
# instruction counts of the hot chains per detail: PMC over the region_debug run (same trace)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc_r04i -o sq --output-format csv -- python3 tools/region_debug.py --config mixed_tenants --batches 5 > gpurun_out/pmc_r04i.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_r04i.log; exit 1; }
grep -E "^batch|hot:" gpurun_out/pmc_r04i.log
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_r04i/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
per = collections.defaultdict(dict)
for r in rows:
    if "k_hot_chains" in r["Kernel_Name"]:
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
for d in sorted(per):
    print(d, {k: "%.4g" % v for k, v in sorted(per[d].items())})
PY
echo done
