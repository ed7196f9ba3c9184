#!/bin/bash
# BERT eager default (finite over 40 steps?), W&D rocprof kernel stats for profiles/.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MIFX_BERT_TRACE=1 timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 40 --warmup 5 > gpurun_out/bert_s2m.log 2>&1 || { echo "bert failed"; tail -30 gpurun_out/bert_s2m.log; exit 1; }
grep "\[bert\] step" gpurun_out/bert_s2m.log | tr '\n' ' ' | cut -c1-300; echo
timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s2m_bench.log 2>&1 || { echo "bert bench failed"; tail -30 gpurun_out/bert_s2m_bench.log; exit 1; }
tail -1 gpurun_out/bert_s2m_bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wd -o wd -- python bench.py --steps 100 --warmup 10 --ref-steps 500 > gpurun_out/prof_wd.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_wd.log; exit 1; }
tail -1 gpurun_out/prof_wd.log | cut -c1-200
