#!/bin/bash
# GPU session H: BN+ReLU kernel rewrite (parallel finalize, register-resident channel params),
# BERT flat-AdamW NaN diagnosis, attention backend microbench, TunableOp trial
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_bn_relu.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_h.log 2>&1 || { tail -60 gpurun_out/pytest_h.log; exit 1; }
tail -1 gpurun_out/pytest_h.log
timeout -k 10 600 python -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_bench.log 2>&1 || { tail -30 gpurun_out/resnet_bench.log; exit 1; }
tail -1 gpurun_out/resnet_bench.log
timeout -k 10 600 python tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady.md 2>gpurun_out/resnet_steady.err || { tail -30 gpurun_out/resnet_steady.err; exit 1; }
head -16 gpurun_out/resnet_steady.md
timeout -k 10 600 python tools/diag_bert_nan.py > gpurun_out/diag_bert.log 2>&1 || { tail -30 gpurun_out/diag_bert.log; exit 1; }
cat gpurun_out/diag_bert.log | grep -v Warning
timeout -k 10 300 python tools/bench_attention.py > gpurun_out/attn.log 2>&1 || { tail -30 gpurun_out/attn.log; exit 1; }
cat gpurun_out/attn.log
timeout -k 10 900 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 --no-flat-adamw --tunable gpurun_out/tunableop_bert.csv > gpurun_out/bert_tunable.log 2>&1 || { tail -30 gpurun_out/bert_tunable.log; exit 1; }
tail -1 gpurun_out/bert_tunable.log
