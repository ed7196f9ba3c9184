#!/bin/bash
# CNN kernels (softmax-CE, LRN, SGD+EMA) + per-layer fused-BN precision diag.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/diag/bn_layer_precision.py > gpurun_out/diag_bn_layers.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/diag_bn_layers.log; exit 1; }
cat gpurun_out/diag_bn_layers.log
timeout -k 10 600 python -u -m pytest tests/test_cnn_ops.py tests/test_pate_training.py tests/test_privacy.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2d.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2d.log; exit 1; }
tail -3 gpurun_out/pytest_s2d.log
