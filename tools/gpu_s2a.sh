#!/bin/bash
# Session-2 re-validation of the restored tree: full GPU suite, smoke, 1-GPU bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_s2a.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_gpu_s2a.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_s2a.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s2a.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke_s2a.log; exit 1; }
cat gpurun_out/smoke_s2a.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s2a.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s2a.log; exit 1; }
tail -1 gpurun_out/bench_s2a.log
