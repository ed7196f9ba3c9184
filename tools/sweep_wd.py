"""W&D fused step time vs batch (tiles per workgroup) and grid: separates the per-tile cost from the
per-launch fixed cost (prologue, slab write, reduce+optimizer)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402


def t_step(batch, grid=None, steps=300):
    tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device="cuda", grid=grid)
    tr.set_data(synthetic_records(1 << 20, device="cuda", seed=1))
    tr.capture()
    for _ in range(20):
        tr.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e6


if __name__ == "__main__":
    for b in (64, 16384, 32768, 65536, 131072, 262144):
        print(json.dumps({"batch": b, "grid": min(b // 64, 256), "us_per_step": round(t_step(b), 2)}), flush=True)
    for g in (64, 128, 192, 256):
        print(json.dumps({"batch": 65536, "grid": g, "us_per_step": round(t_step(65536, g), 2)}), flush=True)
