set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u __graft_entry__.py smoke > gpurun_out/smoke_q.log 2>&1 && tail -1 gpurun_out/smoke_q.log &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_q.log 2>&1; rc=$?; tail -1 gpurun_out/t_q.log; exit $rc
