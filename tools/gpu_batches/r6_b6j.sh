#!/bin/bash
# Round 6, batch 6j: which stream do the DataParallel hooks run on during the captured backward; with the hooks
# pinned to the compute stream, do the coalesced flushes with overlapped exchanges train? Then BERT dX A/B (batch 9).
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
DIAG_STREAMS=1 MIFX_DP_FLUSH_MIN_WG=0 timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 4 > gpurun_out/r6/diag/streams.log 2>&1 || { tail -20 gpurun_out/r6/diag/streams.log; exit 1; }
grep -E "stream|True \[" gpurun_out/r6/diag/streams.log
for t in 1024 2048; do
  MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 8 > gpurun_out/r6/diag/fix_$t.log 2>&1 || { tail -20 gpurun_out/r6/diag/fix_$t.log; exit 1; }
  echo "fixed, min_wg $t: $(tail -1 gpurun_out/r6/diag/fix_$t.log)"
done
bash tools/gpu_batches/r6_b9.sh
