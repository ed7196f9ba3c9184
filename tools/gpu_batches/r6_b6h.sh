#!/bin/bash
# Round 6, batch 6h: coalesced-flush divergence -- is it the IPC exchange or any side-stream in-place work on the
# bucket? MIFX_DP_COMM=copy replaces the exchange by a plain copy out and back on the side stream.
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {
  env "$@" timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 7 > gpurun_out/r6/diag/last.log 2>&1 || { tail -20 gpurun_out/r6/diag/last.log; exit 1; }
  echo "$* -> $(tail -1 gpurun_out/r6/diag/last.log)"
}
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_COMM=copy
run MIFX_DP_FLUSH_MIN_WG=0 MIFX_DP_COMM=copy
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_COMM=side MIFX_DP_FLUSH_LAST=1
echo done
