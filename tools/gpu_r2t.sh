#!/bin/bash
# Round 2: xGMI one-shot DP exchange (2 and 4 processes on one GPU) + W&D regression tests
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2t.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2t.log | tail -30; tail -20 gpurun_out/pytest_r2t.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_r2t.log; tail -1 gpurun_out/pytest_r2t.log
