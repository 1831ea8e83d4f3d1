#!/bin/bash
# round 6: segmented pass-0 output (rl_tune segments: [segment][bin] instead of [bin][tile]) —
# parity, then sw_zipf bench per segment count and scatter0's address-translation misses
set -o pipefail
mkdir -p gpurun_out/r06ac
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_hot.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread -k "segmented or routed or two_pass" > gpurun_out/t_r06ac.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|mismatch" gpurun_out/t_r06ac.log | head; tail -20 gpurun_out/t_r06ac.log; exit 1; }
grep -E "passed|failed" gpurun_out/t_r06ac.log | tail -1
one() {  # tag segs
  timeout -k 10 200 python -u bench.py --config sw_zipf --steps 10 --warmup 3 --no-extra --no-cpu-baseline --tune segments=$2 > gpurun_out/ab.json 2>/dev/null || { echo "bench failed $1"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/ab.json')); s=d['stage_ms']
print('$1 segs=$2', round(d['ms_per_step'],3), 'scatter0', s['scatter0'], 'group', s.get('group'), 'unpermute', s.get('unpermute'), 'region', s['region'], d['status'])"
}
for rep in 1 2; do
  one $rep 1 && one $rep 4 && one $rep 8 && one $rep 16 || exit 1
done
for sg in 8 1; do
  timeout -k 10 -s KILL 120 rocprofv3 --pmc TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum -d gpurun_out/r06ac/s$sg -o s$sg --output-format csv -- python3 bench.py --config sw_zipf --steps 3 --warmup 1 --no-extra --no-cpu-baseline --tune segments=$sg > gpurun_out/r06ac/s$sg.log 2>&1 || { echo "pmc $sg failed"; exit 1; }
  python3 - gpurun_out/r06ac/s$sg <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'scatter_split' in r['Kernel_Name']:
        acc[r['Counter_Name']].append((int(r['Dispatch_Id']), float(r['Counter_Value']), (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3))
for c, v in acc.items():
    v.sort(); print(sys.argv[1][-3:], c, ' '.join(f'{x[1]:.3g}/{x[2]:.0f}us' for x in v))
PY
done
echo done
