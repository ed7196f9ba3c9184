#!/bin/bash
# Round 6, batch 6f: which bucket slots are written after their exchange was launched (tools/dp_late_write_diag.py)
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for t in 1024 0; do
  MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u tools/dp_late_write_diag.py > gpurun_out/r6/diag/late_$t.log 2>&1 || { tail -20 gpurun_out/r6/diag/late_$t.log; exit 1; }
  echo "min_wg $t:"; grep "^step" gpurun_out/r6/diag/late_$t.log
done
echo done
