#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_vocab.py tests/test_pipeline_taxi.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2f.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2f.log; exit 1; }
tail -3 gpurun_out/pytest_s2f.log
timeout -k 10 300 python -u tools/bench_analyzers.py --rows 1048576 > gpurun_out/bench_analyzers.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_analyzers.log; exit 1; }
cat gpurun_out/bench_analyzers.log
timeout -k 10 400 python -u tools/diag/resnet_grad_fp64.py > gpurun_out/diag_resnet_fp64c.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/diag_resnet_fp64c.log; exit 1; }
cat gpurun_out/diag_resnet_fp64c.log
timeout -k 10 600 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 > gpurun_out/bert_s2f.log 2>&1 || { echo "bert failed"; tail -30 gpurun_out/bert_s2f.log; exit 1; }
tail -1 gpurun_out/bert_s2f.log
timeout -k 10 600 python -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_s2f.log 2>&1 || { echo "resnet failed"; tail -30 gpurun_out/resnet_s2f.log; exit 1; }
tail -1 gpurun_out/resnet_s2f.log
