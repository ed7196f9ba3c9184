#!/bin/bash
# BERT default (hipGraph + own-grad FlatAdamW): tests, bench, rocprof of the replayed step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_flat_adamw.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3j.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3j.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_s3j.log
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 50 --warmup 10 > gpurun_out/bert_s3j.log 2>&1 || { echo "bert failed"; tail -12 gpurun_out/bert_s3j.log; exit 1; }
tail -1 gpurun_out/bert_s3j.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert3 -o bert -- python -m mifx.trainer.bert_trainer --steps 40 --warmup 5 > gpurun_out/prof_bert3.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_bert3.log; exit 1; }
find gpurun_out/prof_bert3 -name "*.db"
