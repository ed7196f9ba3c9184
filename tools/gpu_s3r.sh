#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cp profiles/tunableop_bert_base_mi355x.csv gpurun_out/tune_s3r.csv
timeout -k 10 500 python -u -m mifx.trainer.bert_trainer --steps 50 --warmup 10 --tunable gpurun_out/tune_s3r.csv > gpurun_out/bert_s3r.log 2>&1 || { echo "bert failed"; tail -12 gpurun_out/bert_s3r.log; exit 1; }
tail -1 gpurun_out/bert_s3r.log | cut -c1-250
timeout -k 10 500 python -u -m mifx.trainer.bert_trainer --steps 50 --warmup 10 --tunable gpurun_out/tune_s3r.csv > gpurun_out/bert_s3r2.log 2>&1 || { echo "bert2 failed"; tail -12 gpurun_out/bert_s3r2.log; exit 1; }
tail -1 gpurun_out/bert_s3r2.log | cut -c1-250
wc -l gpurun_out/tune_s3r.csv
