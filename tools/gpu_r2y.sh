#!/bin/bash
# Round 2: slab-order optimizer state: W&D + DP GPU tests, A/B timing, DP step overhead, kernel timeline
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2y.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2y.log | tail -30; tail -20 gpurun_out/pytest_r2y.log; exit 1; }
tail -1 gpurun_out/pytest_r2y.log
timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8 --batches 65536,131072,40 --rounds 3 > gpurun_out/ab_r2y.txt 2>&1 || { tail -20 gpurun_out/ab_r2y.txt; exit 1; }
grep config gpurun_out/ab_r2y.txt | grep -v loss
timeout -k 10 300 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead_r2y.jsonl 2> gpurun_out/dp_overhead_r2y.err || { tail -20 gpurun_out/dp_overhead_r2y.err; exit 1; }
grep -E "direct|xgmi" gpurun_out/dp_overhead_r2y.jsonl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_y -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 > gpurun_out/tl_r2y.log 2>&1 || { tail -20 gpurun_out/tl_r2y.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tl_y -name "*.db" | head -1) --last 6 --match wdc_fused,wd_reduce > gpurun_out/timeline_r2y.txt
grep -v columns gpurun_out/timeline_r2y.txt
