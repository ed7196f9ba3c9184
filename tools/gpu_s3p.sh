#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
MIFX_BN_LAYOUT_DIAG=1 timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 1 --warmup 1 --images 512 > gpurun_out/resnet_layout.log 2>&1 || { echo "resnet failed"; tail -12 gpurun_out/resnet_layout.log; exit 1; }
grep "bn-layout" gpurun_out/resnet_layout.log | sort | uniq -c | head -20
