#!/bin/bash
# Round 2: pre-warmed multi-step graph: tests + driver-shaped bench x2 + long bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2n.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2n.log | tail -30; tail -5 gpurun_out/pytest_r2n.log; exit 1; }
tail -1 gpurun_out/pytest_r2n.log
for i in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r2n_$i.json 2> gpurun_out/bench_r2n_$i.err || { tail -20 gpurun_out/bench_r2n_$i.err; exit 1; }
cut -c1-200 gpurun_out/bench_r2n_$i.json
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2n_long.json 2> gpurun_out/bench_r2n_long.err || { tail -20 gpurun_out/bench_r2n_long.err; exit 1; }
cut -c1-200 gpurun_out/bench_r2n_long.json
