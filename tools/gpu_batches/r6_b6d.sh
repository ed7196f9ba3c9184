#!/bin/bash
# Round 6, batch 6d: which part of the coalesced DP flush breaks the captured step -- the final run flushed in the hook
# (MIFX_DP_FLUSH_LAST=1, new default) vs left to the post-backward flush (0); exchanges launched early vs only in
# finish() (MIFX_DP_LAUNCH_LATE=1). Captured steps, B=256, losses per step (tools/dp_flush_diag.py).
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {
  env "$@" timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 7 > gpurun_out/r6/diag/last.log 2>&1 || { tail -20 gpurun_out/r6/diag/last.log; exit 1; }
  echo "$* -> $(tail -1 gpurun_out/r6/diag/last.log)"
}
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_FLUSH_LAST=1
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_FLUSH_LAST=0 MIFX_DP_LAUNCH_LATE=1
run MIFX_DP_FLUSH_MIN_WG=0 MIFX_DP_LAUNCH_LATE=1
run MIFX_DP_FLUSH_MIN_WG=2048 MIFX_DP_FLUSH_LAST=1
echo done
