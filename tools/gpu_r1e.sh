#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_bert_tp.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_bert.log 2>&1 || { tail -40 gpurun_out/pytest_bert.log; exit 1; }
tail -1 gpurun_out/pytest_bert.log
timeout -k 10 600 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 > gpurun_out/bert_bench.log 2>&1 || { tail -30 gpurun_out/bert_bench.log; exit 1; }
tail -1 gpurun_out/bert_bench.log
timeout -k 10 900 python tools/bench_resnet_layout.py > gpurun_out/resnet_layout.log 2>&1 || { tail -30 gpurun_out/resnet_layout.log; exit 1; }
cat gpurun_out/resnet_layout.log | grep format
bash tools/prof_run.sh bert 600 -- python3 -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 5 --warmup 2
