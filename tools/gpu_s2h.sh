#!/bin/bash
# W&D live-granule staging + preloaded tile map; BN fp64 test; BERT replay NaN diag; ResNet bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py tests/test_bn_relu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2h.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2h.log; exit 1; }
tail -3 gpurun_out/pytest_s2h.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s2h.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s2h.log; exit 1; }
tail -1 gpurun_out/bench_s2h.log
timeout -k 10 600 python -u tools/diag/bert_replay_nan.py > gpurun_out/diag_bert_replay.log 2>&1 || { echo "bert diag failed"; tail -30 gpurun_out/diag_bert_replay.log; exit 1; }
cat gpurun_out/diag_bert_replay.log
timeout -k 10 900 python -u -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s2h.log 2>&1 || { echo "resnet failed"; tail -30 gpurun_out/resnet_s2h.log; exit 1; }
tail -4 gpurun_out/resnet_s2h.log
