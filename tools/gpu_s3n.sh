#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_flat_adamw.py tests/test_wide_deep.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3n.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3n.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_s3n.log
