#!/bin/bash
# Round 2: fused attention + W&D L2 ownership: tests, W&D A/B + bench, BERT bench + kernel table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2k.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2k.log | tail -30; tail -5 gpurun_out/pytest_r2k.log; exit 1; }
tail -1 gpurun_out/pytest_r2k.log
timeout -k 10 300 python -u tools/ab_wd.py --kernels chain8,chain4 --batches 65536,40 > gpurun_out/ab_r2k.jsonl 2> gpurun_out/ab_r2k.err || { tail -20 gpurun_out/ab_r2k.err; exit 1; }
cat gpurun_out/ab_r2k.jsonl
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2k.json 2> gpurun_out/bench_r2k.err || { tail -20 gpurun_out/bench_r2k.err; exit 1; }
cat gpurun_out/bench_r2k.json
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_r2k.json 2> gpurun_out/bert_r2k.err || { tail -20 gpurun_out/bert_r2k.err; exit 1; }
tail -1 gpurun_out/bert_r2k.json
timeout -k 10 400 python tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 5 > gpurun_out/bert_steady_r2k.md 2>gpurun_out/bert_steady_r2k.err || { tail -30 gpurun_out/bert_steady_r2k.err; exit 1; }
head -24 gpurun_out/bert_steady_r2k.md
