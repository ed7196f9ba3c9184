#!/bin/bash
# W&D A/B (compact slab x live staging) in one process; vocab kernels after the LDS pre-aggregation;
# BERT main: plain, then with per-step loss trace.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_vocab.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s2i.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s2i.log; exit 1; }
tail -2 gpurun_out/pytest_s2i.log
timeout -k 10 400 python -u tools/ab_wd.py > gpurun_out/ab_wd.log 2>&1 || { echo "ab failed"; tail -30 gpurun_out/ab_wd.log; exit 1; }
cat gpurun_out/ab_wd.log
timeout -k 10 300 python -u tools/bench_analyzers.py --rows 1048576 > gpurun_out/bench_analyzers2.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_analyzers2.log; exit 1; }
cat gpurun_out/bench_analyzers2.log
timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s2i_a.log 2>&1 || { echo "bert a failed"; tail -30 gpurun_out/bert_s2i_a.log; exit 1; }
tail -1 gpurun_out/bert_s2i_a.log
MIFX_BERT_TRACE=1 timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_s2i_b.log 2>&1 || { echo "bert b failed"; tail -30 gpurun_out/bert_s2i_b.log; exit 1; }
grep -v Warning gpurun_out/bert_s2i_b.log | tail -12
