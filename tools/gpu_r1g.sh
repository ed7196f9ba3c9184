#!/bin/bash
# GPU session G: fused BN+ReLU kernels + BERT hipGraph step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_bn_relu.py tests/test_flat_adamw.py tests/test_bert_tp.py -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_g.log 2>&1 || { tail -60 gpurun_out/pytest_g.log; exit 1; }
tail -2 gpurun_out/pytest_g.log
timeout -k 10 600 python -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_bench.log 2>&1 || { tail -30 gpurun_out/resnet_bench.log; exit 1; }
tail -1 gpurun_out/resnet_bench.log
timeout -k 10 600 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 > gpurun_out/bert_bench.log 2>&1 || { tail -30 gpurun_out/bert_bench.log; exit 1; }
tail -1 gpurun_out/bert_bench.log
timeout -k 10 600 python tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady.md 2>gpurun_out/resnet_steady.err || { tail -30 gpurun_out/resnet_steady.err; exit 1; }
head -12 gpurun_out/resnet_steady.md
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
