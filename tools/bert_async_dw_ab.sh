#!/bin/bash
# BERT-base step A/B: weight-gradient GEMMs on a side stream (MIFX_BERT_ASYNC_DW=1) vs in line (0), alternating
# processes; the loss after the same steps must be identical (same kernels, same math, different stream)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for run in 1 2; do
  for v in 1 0; do
    MIFX_BERT_ASYNC_DW=$v timeout -k 10 300 python -u tools/bench_bert.py --steps 30 --warmup 5 > gpurun_out/bert_async_$v$run.log 2>&1 || { tail -20 gpurun_out/bert_async_$v$run.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bert_async_$v$run.log').read().strip().splitlines()[-1]);print('async_dw',$v,'run',$run,round(d['ms_per_step'],3),d['loss'])"
  done
done
