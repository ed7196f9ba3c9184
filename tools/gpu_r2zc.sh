#!/bin/bash
# Round 2: activation gradient overlapped with the staging (before the barrier): tests, A/B, stamps
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2zc.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2zc.log | tail -30; tail -20 gpurun_out/pytest_r2zc.log; exit 1; }
tail -1 gpurun_out/pytest_r2zc.log
timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8,chain4 --batches 65536,131072,40 --rounds 3 > gpurun_out/ab_r2zc.txt 2>&1 || { tail -20 gpurun_out/ab_r2zc.txt; exit 1; }
grep config gpurun_out/ab_r2zc.txt | grep -v loss
timeout -k 10 120 python -u tools/stamps_wdc.py > gpurun_out/stamps_r2zc.txt 2>&1 || { tail -20 gpurun_out/stamps_r2zc.txt; exit 1; }
tail -28 gpurun_out/stamps_r2zc.txt
