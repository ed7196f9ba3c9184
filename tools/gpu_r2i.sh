#!/bin/bash
# Round 2: direct-RCCL data-parallel W&D path: tests + overhead vs split/captured
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2i.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2i.log | tail -30; tail -5 gpurun_out/pytest_r2i.log; exit 1; }
tail -1 gpurun_out/pytest_r2i.log
timeout -k 10 200 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead_r2i.jsonl 2>gpurun_out/dp_overhead_r2i.err || { tail -20 gpurun_out/dp_overhead_r2i.err; exit 1; }
cat gpurun_out/dp_overhead_r2i.jsonl
