#!/bin/bash
# Round 2: W&D step timeline (kernel trace of the captured step) at B=65536 and B=40, chained 8-wave kernel
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for b in 65536 40; do
timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_$b -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches $b --rounds 1 > gpurun_out/tl_$b.log 2>&1 || { tail -20 gpurun_out/tl_$b.log; exit 1; }
python3 tools/timeline.py $(find /tmp/tl_$b -name "*.db" | head -1) --last 8 --match wdc_fused,wd_reduce_opt > gpurun_out/timeline_r2g_$b.txt
cat gpurun_out/timeline_r2g_$b.txt
done
timeout -k 10 200 python -u tools/stamps_wdc.py > gpurun_out/stamps_wdc_r2g.txt 2>&1 || { tail -20 gpurun_out/stamps_wdc_r2g.txt; exit 1; }
tail -25 gpurun_out/stamps_wdc_r2g.txt
