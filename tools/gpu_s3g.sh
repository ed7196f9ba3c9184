#!/bin/bash
# BERT: own-gradient FlatAdamW, bf16-param LN/GELU, HIP bias-grad reductions: tests, bench, steady profile.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_flat_adamw.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3g.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3g.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_s3g.log
MIFX_BERT_TRACE=1 timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s3g.log 2>&1 || { echo "bert failed"; tail -30 gpurun_out/bert_s3g.log; exit 1; }
grep "\[bert\] step" gpurun_out/bert_s3g.log | awk '{print $5}' | tr '\n' ' '; echo
tail -1 gpurun_out/bert_s3g.log | cut -c1-400
timeout -k 10 300 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 5 > gpurun_out/bert_steady_s3g.md 2> gpurun_out/bert_steady_s3g.err || { echo "table failed"; tail -20 gpurun_out/bert_steady_s3g.err; exit 1; }
head -30 gpurun_out/bert_steady_s3g.md | cut -c1-160
