#!/bin/bash
# round 5: hot threshold re-sweep now that the chains start on time and their fill overlaps the
# normal regions (default: max(16384, batch / 4096))
set -o pipefail
mkdir -p gpurun_out
for cfg in sw_zipf zipf_1b mixed_tenants; do
for rep in 1 2; do
for thr in 0 16384 32768 65536 131072; do
T=""; [ $thr != 0 ] && T="--tune hot_threshold=$thr"
timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 3 --no-extra --no-cpu-baseline $T > gpurun_out/b_r05ab.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/b_r05ab.log; exit 1; }
tail -1 gpurun_out/b_r05ab.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d['stage_ms']; print('$cfg thr=$thr', round(d['ms_per_step'],3), 'offs', round(s.get('region_offsets'),3), 'region', round(s.get('region'),3), 'sc1', round(s.get('scatter1'),3), d['status'])"
done
done
done
echo done
