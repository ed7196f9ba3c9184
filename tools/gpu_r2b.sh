#!/bin/bash
# Round 2: validate fused dropout+LN (BERT), shifted-sum BN, pool NaN routing; BERT / ResNet benches.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_bn_relu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2b.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED" gpurun_out/pytest_r2b.log | tail -30; tail -5 gpurun_out/pytest_r2b.log; exit 1; }
tail -2 gpurun_out/pytest_r2b.log
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_r2b.json 2> gpurun_out/bert_r2b.err || { tail -20 gpurun_out/bert_r2b.err; exit 1; }
tail -1 gpurun_out/bert_r2b.json
timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_r2b.json 2> gpurun_out/resnet_r2b.err || { tail -20 gpurun_out/resnet_r2b.err; exit 1; }
tail -1 gpurun_out/resnet_r2b.json
