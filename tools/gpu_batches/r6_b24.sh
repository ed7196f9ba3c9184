#!/bin/bash
# Round 6, batch 24: BERT embedding add + LayerNorm on the fused kernel: tests, step time, aten-op diagnostic.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_bert_tp.py tests/test_bert_component.py tests/test_gemm.py tests/test_tp_ipc.py \
  > gpurun_out/r6/b24_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b24_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b24_tests.log
for i in 1 2 3; do timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 2>/dev/null | grep '^{' | tail -1 | cut -c1-260; done
timeout -k 10 200 python -u tools/bert_misc_diag.py > gpurun_out/r6/bert_misc_diag3.txt 2>&1
head -12 gpurun_out/r6/bert_misc_diag3.txt
echo done
