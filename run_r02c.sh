set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hot.py -q -x --timeout 120 --timeout-method thread > gpurun_out/t_r02c.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/t_r02c.log; exit 1; }
tail -1 gpurun_out/t_r02c.log
for c in tb_uniform mixed_tenants zipf_1b sw_zipf; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/b_r02c_$c.log 2>&1 || { echo "bench $c failed"; tail -5 gpurun_out/b_r02c_$c.log; exit 1; }
  tail -1 gpurun_out/b_r02c_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'frac %.3f'%d['roofline']['frac'], {k:v for k,v in d['stage_ms'].items() if v>0.05})"
done
