#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 50 --warmup 10 > gpurun_out/bert_s3m.log 2>&1 || { echo "bert failed"; tail -12 gpurun_out/bert_s3m.log; exit 1; }
tail -1 gpurun_out/bert_s3m.log | cut -c1-300
timeout -k 10 300 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 5 > gpurun_out/bert_steady_s3m.md 2> gpurun_out/bert_steady_s3m.err || { echo "table failed"; tail -20 gpurun_out/bert_steady_s3m.err; exit 1; }
head -34 gpurun_out/bert_steady_s3m.md | cut -c1-150
