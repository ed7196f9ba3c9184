#!/bin/bash
# BERT NaN bisection on bert_trainer.main: eager+flat, graph+torch AdamW, graph+flat with a seed,
# and the diag path on cuda:0.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export MIFX_BERT_TRACE=1
for v in "--no-graph" "--no-flat-adamw" "--seed 0" "--seed 1" ""; do
  tag=$(echo "x$v" | tr -d ' -')
  timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 12 --warmup 5 $v > gpurun_out/bert_bis_$tag.log 2>&1 || { echo "bert $v failed"; tail -30 gpurun_out/bert_bis_$tag.log; exit 1; }
  echo "== variant '$v':"; grep "\[bert\] step" gpurun_out/bert_bis_$tag.log | tr '\n' ' ' | cut -c1-400; echo
done
