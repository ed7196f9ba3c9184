#!/bin/bash
# Round 2: attention bwd with P_d/dS staged over K/V (2 WG/CU): tests, micro-bench, BERT bench (+ TunableOp A/B)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "attention or bert_hipgraph or finite" > gpurun_out/pytest_r2m.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2m.log | tail -30; tail -5 gpurun_out/pytest_r2m.log; exit 1; }
tail -1 gpurun_out/pytest_r2m.log
timeout -k 10 300 python -u tools/bench_attention.py > gpurun_out/attn_bench_r2m.jsonl 2> gpurun_out/attn_bench_r2m.err || { tail -20 gpurun_out/attn_bench_r2m.err; exit 1; }
cat gpurun_out/attn_bench_r2m.jsonl
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_r2m.json 2> gpurun_out/bert_r2m.err || { tail -20 gpurun_out/bert_r2m.err; exit 1; }
tail -1 gpurun_out/bert_r2m.json
cp profiles/tunableop_bert_base_mi355x.csv /tmp/tunable.csv
timeout -k 10 600 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 --tunable /tmp/tunable.csv > gpurun_out/bert_r2m_tunable.json 2> gpurun_out/bert_r2m_tunable.err || { tail -20 gpurun_out/bert_r2m_tunable.err; exit 1; }
tail -1 gpurun_out/bert_r2m_tunable.json
