#!/bin/bash
# BERT-base training step A/B of the weight-gradient GEMM: hand-written TN kernel on its preferred shapes
# (MIFX_HIP_GEMM_TN=1) vs hipBLASLt (0), alternating, each run its own process; JSON lines appended to
# gpurun_out/bert_tn_ab.jsonl.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for run in 1 2; do
  for tn in 1 0; do
    out=$(MIFX_HIP_GEMM_TN=$tn timeout -k 10 300 python -u tools/bench_bert.py --steps ${1:-30} --warmup 5 2>gpurun_out/bert_tn_err.log | tail -1) || exit 1
    echo "{\"hip_gemm_tn\": $tn, \"run\": $run, \"result\": $out}" | tee -a gpurun_out/bert_tn_ab.jsonl
  done
done
