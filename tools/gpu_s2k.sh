#!/bin/bash
# BERT: tests (incl. main-config finiteness regression), bench, rocprof kernel stats of the graph step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_flat_adamw.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2k.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2k.log; exit 1; }
tail -3 gpurun_out/pytest_s2k.log
timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s2k.log 2>&1 || { echo "bert failed"; tail -30 gpurun_out/bert_s2k.log; exit 1; }
tail -1 gpurun_out/bert_s2k.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o bert -- python -m mifx.trainer.bert_trainer --steps 40 --warmup 5 > gpurun_out/prof_bert.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_bert.log; exit 1; }
find gpurun_out/prof_bert -name "*.db"
