#!/bin/bash
# Round 2, first GPU pass: full GPU test suite, smoke, 1-GPU bench, rocprof of the bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2a.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_r2a.log | tail -20; tail -5 gpurun_out/pytest_r2a.log; exit 1; }
tail -2 gpurun_out/pytest_r2a.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2a.log 2>&1 || { tail -20 gpurun_out/smoke_r2a.log; exit 1; }
tail -1 gpurun_out/smoke_r2a.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 50 --warmup 10 > gpurun_out/bench_r2a.json 2> gpurun_out/bench_r2a.err || { tail -20 gpurun_out/bench_r2a.err; exit 1; }
cat gpurun_out/bench_r2a.json
bash tools/prof_run.sh bench_r2a 300 -- python3 bench.py --gpus 1 --steps 50 --warmup 10
