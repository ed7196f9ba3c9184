#!/bin/bash
# vocab kernels, W&D fixed-point wide-grad determinism, ResNet BN gradient conditioning diag.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_vocab.py tests/test_wide_deep.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2c.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2c.log; exit 1; }
tail -3 gpurun_out/pytest_s2c.log
timeout -k 10 400 python -u tools/diag/resnet_grad_fp64.py > gpurun_out/diag_resnet_fp64b.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/diag_resnet_fp64b.log; exit 1; }
cat gpurun_out/diag_resnet_fp64b.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s2c.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s2c.log; exit 1; }
tail -1 gpurun_out/bench_s2c.log
