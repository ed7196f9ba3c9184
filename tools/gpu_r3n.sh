#!/bin/bash
# ResNet-50 stride-1 3x3 convs on gconv: tests (gconv, BN/ResNet, image pipeline, DP2), ResNet bench A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gconv.py tests/test_bn_relu.py tests/test_image_pipeline.py tests/test_parallel_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rn_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/rn_tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 8 > gpurun_out/rn_bench.json 2> gpurun_out/rn_bench.err || { tail -10 gpurun_out/rn_bench.err; exit 1; }
tail -1 gpurun_out/rn_bench.json
