#!/bin/bash
# Round 2: slab reduction variants: XCD-local (default), plain one-pass, one-pass with nontemporal / agent-scope loads
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in xcd plain; do
  unset MIFX_WD_XCD MIFX_LIB_WIDE_DEEP
  case $v in plain) export MIFX_WD_XCD=0;; nt) export MIFX_WD_XCD=0 MIFX_LIB_WIDE_DEEP=$PWD/tools/bin/libwd_sl1.so;; agent) export MIFX_WD_XCD=0 MIFX_LIB_WIDE_DEEP=$PWD/tools/bin/libwd_sl2.so;; esac
  timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 3 > gpurun_out/ab_r2za_$v.txt 2>&1 || { tail -20 gpurun_out/ab_r2za_$v.txt; exit 1; }
  echo "== $v"; grep config gpurun_out/ab_r2za_$v.txt | grep -v loss
  timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/tl_za_$v -o tl -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 > gpurun_out/tl_r2za_$v.log 2>&1 || { tail -20 gpurun_out/tl_r2za_$v.log; exit 1; }
  python3 tools/timeline.py $(find /tmp/tl_za_$v -name "*.db" | head -1) --last 4 --match wdc_fused,wd_reduce,wd_xcd > gpurun_out/timeline_r2za_$v.txt
  grep -v columns gpurun_out/timeline_r2za_$v.txt
done
