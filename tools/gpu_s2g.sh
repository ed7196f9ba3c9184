#!/bin/bash
# W&D compact slab (tests + bench), BERT mode diag, ResNet bench with progress, updated BN test.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py tests/test_cnn_ops.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2g.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2g.log; exit 1; }
tail -3 gpurun_out/pytest_s2g.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s2g.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s2g.log; exit 1; }
tail -1 gpurun_out/bench_s2g.log
timeout -k 10 600 python -u tools/diag/bert_modes.py > gpurun_out/diag_bert_modes.log 2>&1 || { echo "bert diag failed"; tail -30 gpurun_out/diag_bert_modes.log; exit 1; }
cat gpurun_out/diag_bert_modes.log
timeout -k 10 900 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s2g.log 2>&1 || { echo "resnet failed"; tail -30 gpurun_out/resnet_s2g.log; exit 1; }
tail -4 gpurun_out/resnet_s2g.log
