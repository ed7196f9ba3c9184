#!/bin/bash
# ResNet-50 step A/B of the BN stats kernel: current build vs tools/bin/libbn_relu_old.so (MIFX_LIB_BN_RELU),
# alternating; each run streams its output to gpurun_out/ab_bn_<variant><run>.log (no silent stretches)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for run in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export MIFX_LIB_BN_RELU=$PWD/tools/bin/libbn_relu_old.so; else unset MIFX_LIB_BN_RELU; fi
    echo "[ab_bn] $v $run start"
    timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 > gpurun_out/ab_bn_$v$run.log 2>&1 || exit 1
    echo "$v $run $(tail -1 gpurun_out/ab_bn_$v$run.log | cut -c1-220)"
  done
done
