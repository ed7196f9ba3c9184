#!/bin/bash
# BERT eager default step: steady-state kernel table.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 5 > gpurun_out/bert_steady_s3.md 2> gpurun_out/bert_steady_s3.err || { echo "table failed"; tail -20 gpurun_out/bert_steady_s3.err; exit 1; }
head -40 gpurun_out/bert_steady_s3.md | cut -c1-200
