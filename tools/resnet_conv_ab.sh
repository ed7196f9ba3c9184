#!/bin/bash
# Whole-step A/B of ResNet-50 (B=256, bf16) with the block convs on MIOpen (0) vs csrc/gconv.hip (1), alternating
# runs in fresh processes: tools/resnet_conv_ab.sh [steps] -> gpurun_out/resnet_ab.jsonl (one line per run; the
# runs' logs stream into gpurun_out/resnet_ab_<h>_<i>.log)
set -o pipefail
steps=${1:-40}
mkdir -p gpurun_out
for i in 1 2; do
  for h in 0 1; do
    log=gpurun_out/resnet_ab_${h}_${i}.log
    MIFX_RESNET_HIP_CONV=$h timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps "$steps" > "$log" 2>&1 || exit 1
    echo "{\"hip_conv\": $h, \"run\": $i, \"result\": $(grep '^{' "$log" | tail -1)}" >> gpurun_out/resnet_ab.jsonl
  done
done
cat gpurun_out/resnet_ab.jsonl
