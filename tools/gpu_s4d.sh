#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_bn_relu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s4d.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s4d.log | tail -20; exit 1; }
tail -2 gpurun_out/pytest_s4d.log
timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s4d.log 2>&1 || { echo "resnet failed"; tail -20 gpurun_out/resnet_s4d.log; exit 1; }
tail -1 gpurun_out/resnet_s4d.log
timeout -k 10 400 python tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady_s4d.md 2>gpurun_out/resnet_steady_s4d.err || { tail -30 gpurun_out/resnet_steady_s4d.err; exit 1; }
grep -E "GPU time|finalize|bn_" gpurun_out/resnet_steady_s4d.md
