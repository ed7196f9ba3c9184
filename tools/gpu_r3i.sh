#!/bin/bash
# TF-SAME NHWC max-pool kernels: pool tests, ResNet/PATE tests, PATE bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_bn_relu.py tests/test_cnn_ops.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pool_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/pool_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_pate.py --steps 30 > gpurun_out/pate_bench4.jsonl 2> gpurun_out/pate_bench4.err || { tail -20 gpurun_out/pate_bench4.err; exit 1; }
cat gpurun_out/pate_bench4.jsonl
