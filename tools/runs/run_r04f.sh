#!/bin/bash
# window of 1 chunk (the round-3 structure after the clean-up): region timeline of mixed over 6
# batches, then one PMC pass of instruction counters over a mixed bench run (hot chains' share)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/region_debug.py --config mixed_tenants --batches 6 > gpurun_out/rd_r04f.log 2>&1 || { echo "region_debug failed"; tail -20 gpurun_out/rd_r04f.log; exit 1; }
grep -E "^batch|dur" gpurun_out/rd_r04f.log | tail -14
timeout -k 10 -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc_r04f -o sq --output-format csv -- python3 bench.py --config mixed_tenants --steps 2 --warmup 4 --no-cpu-baseline --no-extra > gpurun_out/pmc_r04f.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_r04f.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_r04f/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in rows:
    k = r["Kernel_Name"].split("(")[0][:60]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, v in sorted(agg.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0))[:8]:
    n = len(disp[k])
    print(k, n, {c: "%.3g" % (x / n) for c, x in sorted(v.items())})
PY
echo done
