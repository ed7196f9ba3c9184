#!/bin/bash
# Round 2: per-block clock stamps of the chained kernel + kernel-trace timeline of the captured step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python -u tools/stamps_wdc.py > gpurun_out/stamps_r2p.txt 2>&1 || { tail -20 gpurun_out/stamps_r2p.txt; exit 1; }
tail -12 gpurun_out/stamps_r2p.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_r2p -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 > gpurun_out/tl_r2p.log 2>&1 || { tail -20 gpurun_out/tl_r2p.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tl_r2p -name "*.db" | head -1) --last 8 --match wdc_fused,wd_reduce_opt > gpurun_out/timeline_r2p.txt
cat gpurun_out/timeline_r2p.txt
