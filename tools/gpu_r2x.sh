#!/bin/bash
# Round 2: kernel timeline of the 1-rank xGMI DP step vs the direct RCCL step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in xgmi direct; do
timeout -k 10 150 rocprofv3 --kernel-trace -d /tmp/tl_x_$m -o tl -- python3 tools/dp_step_overhead.py $m > gpurun_out/tl_r2x_$m.log 2>&1 || { tail -20 gpurun_out/tl_r2x_$m.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tl_x_$m -name "*.db" | head -1) --last 12 --match wdc_fused,wd_reduce,wd_xgmi,ncclDevKernel,Kernel_Sum > gpurun_out/timeline_r2x_$m.txt
echo "== $m"; grep us_per_step gpurun_out/tl_r2x_$m.log | cut -c1-160; cat gpurun_out/timeline_r2x_$m.txt | grep -v columns
done
