#!/bin/bash
# Round-end rehearsal: full GPU suite, smoke, headline bench (as the driver runs them).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_s4b.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu_s4b.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_gpu_s4b.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s4b.log 2>&1 || { echo smoke failed; tail -30 gpurun_out/smoke_s4b.log; exit 1; }
tail -3 gpurun_out/smoke_s4b.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s4b.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s4b.log; exit 1; }
tail -1 gpurun_out/bench_s4b.log
