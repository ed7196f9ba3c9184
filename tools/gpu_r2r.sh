#!/bin/bash
# Round 2: A/B nontemporal slab stores (tools/bin/libwdc_nt.so) vs production chained kernel, with kernel traces
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base nt; do
  if [ $v = nt ]; then export MIFX_LIB_WD_CHAIN=$PWD/tools/bin/libwdc_nt.so; fi
  timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8 --batches 65536,131072 --rounds 3 > gpurun_out/ab_r2r_$v.txt 2>&1 || { tail -20 gpurun_out/ab_r2r_$v.txt; exit 1; }
  grep -v loss gpurun_out/ab_r2r_$v.txt
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_r2r_$v -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 > gpurun_out/tl_r2r_$v.log 2>&1 || { tail -20 gpurun_out/tl_r2r_$v.log; exit 1; }
  python3 tools/timeline.py $(find /tmp/tl_r2r_$v -name "*.db" | head -1) --last 6 --match wdc_fused,wd_reduce_opt > gpurun_out/timeline_r2r_$v.txt
  cat gpurun_out/timeline_r2r_$v.txt
done
