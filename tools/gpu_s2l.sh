#!/bin/bash
# BERT NaN bisection, 40 timed steps each, per-step loss trace.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, env, args
  local tag=$1; shift; local envs=$1; shift
  env $envs MIFX_BERT_TRACE=1 timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 40 --warmup 5 "$@" > gpurun_out/bert_l_$tag.log 2>&1 || { echo "bert $tag failed"; tail -20 gpurun_out/bert_l_$tag.log; exit 1; }
  echo "== $tag: first NaN at step: $(grep -n 'loss nan' gpurun_out/bert_l_$tag.log | head -1 | cut -d' ' -f3) ; last: $(grep '\[bert\] step' gpurun_out/bert_l_$tag.log | tail -1)"
}
run graph_torchadamw "X=1"
run eager_flat "X=1" --no-graph
run eager_torch "X=1" --no-graph --no-flat-adamw
run graph_sync "MIFX_BERT_SYNC=1"
run graph_nodropout "X=1" --dropout 0.0
