#!/bin/bash
# GPU validation: tests, smoke, bench, rocprof summary. Each GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 400 python bench.py --steps 200 --warmup 20 > gpurun_out/bench.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o wd -- python bench.py --steps 50 --warmup 5 --ref-steps 200 > gpurun_out/prof_bench.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_bench.log; exit 1; }
find gpurun_out/prof -name "*stats*" | head
