#!/bin/bash
# Round 2: fused attention kernels (numerics), BERT bench with them, steady-state kernel table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2j.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2j.log | tail -30; tail -5 gpurun_out/pytest_r2j.log; exit 1; }
tail -1 gpurun_out/pytest_r2j.log
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_r2j.json 2> gpurun_out/bert_r2j.err || { tail -20 gpurun_out/bert_r2j.err; exit 1; }
tail -1 gpurun_out/bert_r2j.json
timeout -k 10 400 python tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 5 > gpurun_out/bert_steady_r2j.md 2>gpurun_out/bert_steady_r2j.err || { tail -30 gpurun_out/bert_steady_r2j.err; exit 1; }
head -24 gpurun_out/bert_steady_r2j.md
