#!/bin/bash
# Round 2: chained W&D kernel, 4- vs 8-wave shapes: numerics, A/B timing, phase stamps
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2e.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2e.log | tail -30; tail -5 gpurun_out/pytest_r2e.log; exit 1; }
tail -2 gpurun_out/pytest_r2e.log
timeout -k 10 300 python -u tools/ab_wd.py > gpurun_out/ab_r2e.jsonl 2> gpurun_out/ab_r2e.err || { tail -20 gpurun_out/ab_r2e.err; exit 1; }
cat gpurun_out/ab_r2e.jsonl
timeout -k 10 200 python -u tools/stamps_wdc.py > gpurun_out/stamps_wdc_r2e.txt 2>&1 || { tail -20 gpurun_out/stamps_wdc_r2e.txt; exit 1; }
cat gpurun_out/stamps_wdc_r2e.txt
