#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 > gpurun_out/bert_bench.log 2>&1 || { tail -30 gpurun_out/bert_bench.log; exit 1; }
tail -1 gpurun_out/bert_bench.log
timeout -k 10 600 python -m mifx.trainer.resnet_trainer --batch 256 --images 2048 --steps 20 --warmup 5 > gpurun_out/resnet_bench.log 2>&1 || { tail -30 gpurun_out/resnet_bench.log; exit 1; }
tail -1 gpurun_out/resnet_bench.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert2 -o bert -- python3 -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 5 --warmup 2 > gpurun_out/prof_bert.log 2>&1 || { tail -20 gpurun_out/prof_bert.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet -o resnet -- python3 -m mifx.trainer.resnet_trainer --batch 256 --images 1024 --steps 5 --warmup 2 > gpurun_out/prof_resnet.log 2>&1 || { tail -20 gpurun_out/prof_resnet.log; exit 1; }
echo prof ok
