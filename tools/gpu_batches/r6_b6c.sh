#!/bin/bash
# Round 6, batch 6c: coalesced DP flush divergence at B=256 -- eager and captured losses per threshold, and the first
# captured step's gradients diffed across thresholds (tools/dp_flush_diag.py).
set -o pipefail
mkdir -p gpurun_out/r6/diag
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for t in 0 1024 100000; do
  MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/diag_e$t.pt --steps 3 > gpurun_out/r6/diag/e$t.log 2>&1 || { tail -20 gpurun_out/r6/diag/e$t.log; exit 1; }
  tail -1 gpurun_out/r6/diag/e$t.log
  MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u tools/dp_flush_diag.py /tmp/diag_g$t.pt --graph --steps 6 > gpurun_out/r6/diag/g$t.log 2>&1 || { tail -20 gpurun_out/r6/diag/g$t.log; exit 1; }
  tail -1 gpurun_out/r6/diag/g$t.log
done
python - <<'PY' > gpurun_out/r6/diag/diff.txt
import torch
for mode in ("e", "g"):
    ref = torch.load(f"/tmp/diag_{mode}0.pt", weights_only=True)
    for t in (1024, 100000):
        d = torch.load(f"/tmp/diag_{mode}{t}.pt", weights_only=True)
        bad = []
        for n, g in ref["grads"].items():
            h = d["grads"][n]
            rel = float((g - h).norm() / (g.norm() + 1e-30))
            if rel > 1e-3 or not torch.isfinite(h).all():
                bad.append((n, rel))
        print(mode, t, "losses", d["losses"], "vs", ref["losses"], "params differing:", len(bad), bad[:12])
PY
cat gpurun_out/r6/diag/diff.txt
echo done
