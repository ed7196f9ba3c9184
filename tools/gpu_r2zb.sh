#!/bin/bash
# Round 2: xGMI DP with the XCD-local local sum: DP tests, 1-GPU DP overhead, W&D tests
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_wide_deep.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2zb.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2zb.log | tail -30; tail -20 gpurun_out/pytest_r2zb.log; exit 1; }
grep -c PASSED gpurun_out/pytest_r2zb.log; tail -1 gpurun_out/pytest_r2zb.log
timeout -k 10 300 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead_r2zb.jsonl 2> gpurun_out/dp_overhead_r2zb.err || { tail -20 gpurun_out/dp_overhead_r2zb.err; exit 1; }
grep -E "direct|xgmi" gpurun_out/dp_overhead_r2zb.jsonl
