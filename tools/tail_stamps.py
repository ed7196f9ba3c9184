"""Phase timing of the one-launch W&D step (csrc/wd_chain.hip TailArgs.dbg): per-workgroup real-time stamps
(100 MHz) at kernel start, end of the iterations, barrier 1 passed, level 1 done, barrier 2 passed, end; prints
percentiles over the workgroups of one launch (relative to the earliest start)."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402

batch = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device="cuda", in_kernel_tail=True)
tr.set_data(synthetic_records(1 << 20, device="cuda", seed=1))
tr._ktail.dbg = torch.zeros(256, 8, dtype=torch.int64, device="cuda")
for _ in range(20):
    tr.step()
torch.cuda.synchronize()
d = tr._ktail.dbg[:tr.grid, :6].cpu().numpy().astype(np.float64)
d = (d - d[:, 0].min()) / 100.0  # us
names = ["start", "iters done", "barrier1 passed", "level1 done", "barrier2 passed", "end"]
out = {}
for i, n in enumerate(names):
    out[n] = [round(float(np.percentile(d[:, i], q)), 2) for q in (0, 10, 50, 90, 100)]
print(json.dumps({"batch": batch, "grid": tr.grid, "us_percentiles_0_10_50_90_100": out}))
