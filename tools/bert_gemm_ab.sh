#!/bin/bash
# BERT-base training step A/B: hand-written GEMM on its preferred shapes (MIFX_BERT_HIP_GEMM=1) vs all-hipBLASLt (0),
# alternating, each run its own process; JSON lines appended to gpurun_out/bert_gemm_ab.jsonl.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for run in 1 2; do
  for hip in 1 0; do
    out=$(MIFX_BERT_HIP_GEMM=$hip timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps ${1:-30} --warmup 5 2>gpurun_out/bert_ab_err.log | tail -1) || exit 1
    echo "{\"hip_gemm\": $hip, \"run\": $run, \"result\": $out}" | tee -a gpurun_out/bert_gemm_ab.jsonl
  done
done
