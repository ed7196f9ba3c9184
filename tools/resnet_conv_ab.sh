#!/bin/bash
# Whole-step A/B of ResNet-50 (B=256, bf16) with the block convs on MIOpen (0) vs csrc/gconv.hip (1), alternating
# runs in fresh processes: tools/resnet_conv_ab.sh [steps]  -> one JSON line per run (hip_conv tagged)
set -o pipefail
steps=${1:-40}
for i in 1 2; do
  for h in 0 1; do
    out=$(MIFX_RESNET_HIP_CONV=$h timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps "$steps" 2>/dev/null | tail -1) || exit 1
    echo "{\"hip_conv\": $h, \"run\": $i, \"result\": $out}"
  done
done
