#!/bin/bash
# Round 6, batch 6i: does anything EXECUTE during the capture of the coalesced DP step (weights / gradients changed
# by tr._capture() alone)? Then the W&D data-parallel bench rehearsal on the shared GPU (2 and 4 ranks).
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for t in 1024 0; do
  DIAG_CAPTURE_CHECK=1 MIFX_DP_FLUSH_MIN_WG=$t MIFX_DP_COMM=copy timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 3 > gpurun_out/r6/diag/cap_$t.log 2>&1 || { tail -20 gpurun_out/r6/diag/cap_$t.log; exit 1; }
  echo "min_wg $t:"; grep -E "changed|True \[" gpurun_out/r6/diag/cap_$t.log
done
bash tools/bench_shared_rehearsal.sh 2 || exit 1
bash tools/bench_shared_rehearsal.sh 4 || exit 1
echo done
