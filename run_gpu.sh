#!/bin/bash
# GPU-box driver for one iteration: smoke, GPU parity tests, 1-GPU bench.
# usage: bash run_gpu.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-x}; shift
mkdir -p gpurun_out
timeout -k 10 150 python -u __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 || { echo "smoke failed rc=$?"; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1; echo "bench rc=$?"
tail -1 gpurun_out/bench_$TAG.log
