#!/bin/bash
# Round 2: W&D reduce_opt with 8-column workgroups: tests, bench, timeline
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2l.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2l.log | tail -30; tail -5 gpurun_out/pytest_r2l.log; exit 1; }
tail -1 gpurun_out/pytest_r2l.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2l.json 2> gpurun_out/bench_r2l.err || { tail -20 gpurun_out/bench_r2l.err; exit 1; }
cat gpurun_out/bench_r2l.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tlb -o tl -- python3 bench.py --gpus 1 --steps 50 --warmup 10 --ref-batch 0 > gpurun_out/tlb_r2l.log 2>&1 || { tail -20 gpurun_out/tlb_r2l.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tlb -name "*.db" | head -1) --last 4 --match wdc_fused,wd_reduce_opt
