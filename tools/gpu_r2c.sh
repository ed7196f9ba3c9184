#!/bin/bash
# Round 2: validate the register-chained W&D kernel (numerics vs torch and vs the tile kernel), A/B timing.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2c.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2c.log | tail -30; tail -5 gpurun_out/pytest_r2c.log; exit 1; }
tail -2 gpurun_out/pytest_r2c.log
timeout -k 10 300 python -u tools/ab_wd.py > gpurun_out/ab_r2c.jsonl 2> gpurun_out/ab_r2c.err || { tail -20 gpurun_out/ab_r2c.err; exit 1; }
cat gpurun_out/ab_r2c.jsonl
