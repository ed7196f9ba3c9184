#!/bin/bash
# Round 6, batch 6k: coalesced DP flushes with ONE fork of the communication stream per batch of launches (instead
# of one wait per bucket): captured B=256 losses, and the forced-DP throughput if it trains.
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
run() {
  env "$@" timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/d.pt --graph --steps 8 > gpurun_out/r6/diag/last.log 2>&1 || { tail -20 gpurun_out/r6/diag/last.log; exit 1; }
  echo "$* -> $(tail -1 gpurun_out/r6/diag/last.log)"
}
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_FORK_ONCE=1
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_FORK_ONCE=0
run MIFX_DP_FLUSH_MIN_WG=1024 MIFX_DP_FORK_ONCE=1 MIFX_DP_COMM=copy
for t in 1024 2048; do
  MIFX_DP_FORCE=1 MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 25 --warmup 5 > gpurun_out/r6/resnet_dpf_fo_$t.json 2> gpurun_out/r6/resnet_dpf_fo_$t.err || { tail -20 gpurun_out/r6/resnet_dpf_fo_$t.err; exit 1; }
  echo "min_wg $t fork-once: $(grep '^{' gpurun_out/r6/resnet_dpf_fo_$t.json | tail -1 | cut -c1-200)"
done
echo done
