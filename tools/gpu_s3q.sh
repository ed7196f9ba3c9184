#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bn_relu.py tests/test_image_pipeline.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3q.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3q.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_s3q.log
timeout -k 10 500 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_s3q.log 2>&1 || { echo "resnet failed"; tail -12 gpurun_out/resnet_s3q.log; exit 1; }

tail -1 gpurun_out/resnet_s3q.log | cut -c1-200
