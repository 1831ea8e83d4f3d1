set -o pipefail
timeout -k 10 150 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; exit 1; }
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
