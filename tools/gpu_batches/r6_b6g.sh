#!/bin/bash
# Round 6, batch 6g: coalesced-flush divergence -- split-wait vs three-kernel exchange; bigger / smaller buckets.
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {
  env "$@" timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 7 > gpurun_out/r6/diag/last.log 2>&1 || { tail -20 gpurun_out/r6/diag/last.log; exit 1; }
  echo "$* -> $(tail -1 gpurun_out/r6/diag/last.log)"
}
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_WAITERS=0
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_WAITERS=1
run MIFX_DP_FLUSH_MIN_WG=0 MIFX_DP_WAITERS=1 MIFX_DP_BUCKET_MB=4
echo done
