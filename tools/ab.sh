# usage: bash tools/ab.sh "<variants>"   (GPU box) — parity tests, then interleaved variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ab.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ablate.py --rounds 5 --variants "$1" 2>&1 | tee gpurun_out/ablate.log
