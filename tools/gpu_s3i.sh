#!/bin/bash
# Graph-safe embedding backward: replay diagnostics, graph vs eager BERT steps, tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0


MIFX_BERT_TRACE=1 timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 40 --warmup 5 --graph > gpurun_out/bert_s3i_graph.log 2>&1 || { echo "bert graph failed"; grep -v "^frame" gpurun_out/bert_s3i_graph.log | tail -12; exit 1; }
grep "\[bert\] step" gpurun_out/bert_s3i_graph.log | awk '{print $5}' | tr '\n' ' '; echo
tail -1 gpurun_out/bert_s3i_graph.log | cut -c1-330
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s3i_eager.log 2>&1 || { echo "bert eager failed"; tail -12 gpurun_out/bert_s3i_eager.log; exit 1; }
tail -1 gpurun_out/bert_s3i_eager.log | cut -c1-330
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_flat_adamw.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3i.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3i.log | tail -30; exit 1; }
tail -2 gpurun_out/pytest_s3i.log
