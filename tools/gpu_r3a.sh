#!/bin/bash
# new multi-rank GPU rehearsal tests (BERT TP=2, ResNet-50 DP=2 on one device over gloo)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_parallel_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/par_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|assert|^E " gpurun_out/par_gpu.log | tail -40
exit $rc
