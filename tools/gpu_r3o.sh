#!/bin/bash
# ResNet-50 A/B: stride-1 3x3 convs on gconv vs MIOpen, alternating runs
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 0 1 0 1; do
  MIFX_RESNET_HIP_CONV=$v timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 40 --warmup 10 > gpurun_out/rn_ab_$v.json 2> gpurun_out/rn_ab_$v.err || { tail -10 gpurun_out/rn_ab_$v.err; exit 1; }
  echo "hip_conv=$v $(tail -1 gpurun_out/rn_ab_$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), "img/s", round(d["ms_per_step"],2), "ms")')"
done
