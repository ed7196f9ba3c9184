#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_s3o.log 2>&1 || { echo "resnet failed"; tail -12 gpurun_out/resnet_s3o.log; exit 1; }
tail -1 gpurun_out/resnet_s3o.log | cut -c1-300
timeout -k 10 400 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady_s3o.md 2> gpurun_out/resnet_steady_s3o.err || { echo "table failed"; tail -20 gpurun_out/resnet_steady_s3o.err; exit 1; }
head -40 gpurun_out/resnet_steady_s3o.md | cut -c1-150
