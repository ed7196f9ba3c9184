#!/bin/bash
# Round 6, batch 10: the 8-rank bench.py flow rehearsed on one GPU (W&D DP over the xGMI exchange; timings
# meaningless), and the BERT trainer at TP=4 with sequence parallelism via torchrun (ranks sharing the GPU).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
bash tools/bench_shared_rehearsal.sh 8 || exit 1
MIFX_SHARED_GPU=1 MIFX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29631 -m mifx.trainer.bert_trainer --layers 2 --steps 10 --warmup 3 \
  --sequence-parallel > gpurun_out/r6/bert_tp4_sp.json 2> gpurun_out/r6/bert_tp4_sp.err || { tail -20 gpurun_out/r6/bert_tp4_sp.err; exit 1; }
grep '^{' gpurun_out/r6/bert_tp4_sp.json | tail -1 | cut -c1-300
echo done
