#!/bin/bash
# round 6: scatter0's two modes vs address translation: UTCL1 requests / misses per run
set -o pipefail
mkdir -p gpurun_out/r06z
export TMPDIR=/tmp
for k in 1 2 3 4 5; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum -d gpurun_out/r06z/p$k -o p$k --output-format csv -- python3 bench.py --config sw_zipf --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/r06z/p$k.log 2>&1 || { echo "pmc run $k failed"; exit 1; }
  python3 - gpurun_out/r06z/p$k <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r['Kernel_Name']
    if 'scatter_split' in k or 'gplace' in k or 'unpermute_split' in k:
        acc[k[:40]][r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value']), int(r['End_Timestamp']) - int(r['Start_Timestamp'])))
for k, d in acc.items():
    for c, v in d.items():
        v.sort()
        print(sys.argv[1][-2:], k, c, ' '.join(f'{x[1]:.3g}/{x[2]/1e3:.0f}us' for x in v))
PY
done
echo done
