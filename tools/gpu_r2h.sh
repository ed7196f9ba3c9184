#!/bin/bash
# Round 2: multi-step hipGraph W&D step: test, bench, timeline
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "multi_step or converges or deterministic" > gpurun_out/pytest_r2h.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2h.log | tail -30; tail -5 gpurun_out/pytest_r2h.log; exit 1; }
tail -1 gpurun_out/pytest_r2h.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2h.json 2> gpurun_out/bench_r2h.err || { tail -20 gpurun_out/bench_r2h.err; exit 1; }
cat gpurun_out/bench_r2h.json
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r2h_driver.json 2> gpurun_out/bench_r2h_driver.err || { tail -20 gpurun_out/bench_r2h_driver.err; exit 1; }
cat gpurun_out/bench_r2h_driver.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tlb -o tl -- python3 bench.py --gpus 1 --steps 50 --warmup 10 --ref-batch 0 > gpurun_out/tlb.log 2>&1 || { tail -20 gpurun_out/tlb.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tlb -name "*.db" | head -1) --last 8 --match wdc_fused,wd_reduce_opt > gpurun_out/timeline_r2h.txt
python3 tools/prof_summary.py $(find /tmp/tlb -name "*.db" | head -1) --out gpurun_out/bench_r2h_kernels.md > /dev/null
cat gpurun_out/timeline_r2h.txt
head -8 gpurun_out/bench_r2h_kernels.md
