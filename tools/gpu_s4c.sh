#!/bin/bash
# MIOpen find mode A/B for the ResNet-50 trainer (default dynamic-hybrid vs NORMAL full search).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s4c_default.log 2>&1 || { echo "default failed"; tail -20 gpurun_out/resnet_s4c_default.log; exit 1; }
tail -1 gpurun_out/resnet_s4c_default.log | cut -c1-220
MIOPEN_FIND_MODE=1 timeout -k 10 700 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s4c_normal.log 2>&1 || { echo "normal failed"; tail -20 gpurun_out/resnet_s4c_normal.log; exit 1; }
tail -1 gpurun_out/resnet_s4c_normal.log | cut -c1-220
