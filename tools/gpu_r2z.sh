#!/bin/bash
# Round 2: XCD-local two-level slab reduction: W&D GPU tests, A/B timing, kernel timeline, bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2z.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2z.log | tail -30; tail -20 gpurun_out/pytest_r2z.log; exit 1; }
tail -1 gpurun_out/pytest_r2z.log
timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8 --batches 65536,131072,40 --rounds 3 > gpurun_out/ab_r2z.txt 2>&1 || { tail -20 gpurun_out/ab_r2z.txt; exit 1; }
grep config gpurun_out/ab_r2z.txt | grep -v loss
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_z -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 > gpurun_out/tl_r2z.log 2>&1 || { tail -20 gpurun_out/tl_r2z.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tl_z -name "*.db" | head -1) --last 9 --match wdc_fused,wd_reduce,wd_xcd > gpurun_out/timeline_r2z.txt
grep -v columns gpurun_out/timeline_r2z.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2z.json 2> gpurun_out/bench_r2z.err || { tail -20 gpurun_out/bench_r2z.err; exit 1; }
cut -c1-200 gpurun_out/bench_r2z.json
