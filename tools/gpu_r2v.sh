#!/bin/bash
# Round 2: xGMI DP tests + 1-GPU DP step overhead per exchange path (incl. xgmi) + bench at N=1
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2v.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2v.log | tail -30; tail -20 gpurun_out/pytest_r2v.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_r2v.log; tail -1 gpurun_out/pytest_r2v.log
timeout -k 10 300 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead_r2v.jsonl 2> gpurun_out/dp_overhead_r2v.err || { tail -20 gpurun_out/dp_overhead_r2v.err; exit 1; }
cat gpurun_out/dp_overhead_r2v.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2v.json 2> gpurun_out/bench_r2v.err || { tail -20 gpurun_out/bench_r2v.err; exit 1; }
cut -c1-240 gpurun_out/bench_r2v.json
