#!/bin/bash
# Round-end rehearsal: the driver's GPU tiers (full GPU test suite, smoke, 1-GPU bench with its default flags)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1050 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rehearsal.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_rehearsal.log | tail -30; tail -5 gpurun_out/pytest_rehearsal.log; exit 1; }
tail -1 gpurun_out/pytest_rehearsal.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_rehearsal.log 2>&1 || { tail -20 gpurun_out/smoke_rehearsal.log; exit 1; }
tail -1 gpurun_out/smoke_rehearsal.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_rehearsal.json 2> gpurun_out/bench_rehearsal.err || { tail -20 gpurun_out/bench_rehearsal.err; exit 1; }
cat gpurun_out/bench_rehearsal.json
# configs 4 / 5 on the same box (after the driver tiers)
if [ "${REHEARSAL_CONFIGS:-0}" = "1" ]; then
  timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_rehearsal.json 2> gpurun_out/bert_rehearsal.err || { tail -20 gpurun_out/bert_rehearsal.err; exit 1; }
  grep '^{' gpurun_out/bert_rehearsal.json | tail -1
  timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_rehearsal.json 2> gpurun_out/resnet_rehearsal.err || { tail -20 gpurun_out/resnet_rehearsal.err; exit 1; }
  grep '^{' gpurun_out/resnet_rehearsal.json | tail -1
fi
