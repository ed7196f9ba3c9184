"""Time the KFP taxi DNN trainer (hidden 1500, Adagrad lr 0.1, B=32 reference config and a larger B)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.models.taxi_dnn import TaxiDNN, TaxiDNNConfig  # noqa: E402
from mifx.trainer.taxi_dnn_trainer import TaxiDNNTrainer  # noqa: E402


def run(device, batch, steps, warmup):
    cfg = TaxiDNNConfig()
    g = torch.Generator().manual_seed(0)
    n = max(batch * 64, 10000)
    ids = torch.stack([torch.randint(0, s, (n,), generator=g) for _, s in cfg.sparse], 1)
    dense = torch.randn(n, 3, generator=g)
    y = (torch.rand(n, generator=g) < 0.3).float()
    tr = TaxiDNNTrainer(TaxiDNN(cfg, seed=0), batch=batch, device=device)
    tr.set_data(ids, dense, y)
    tr.run(warmup)
    if device != "cpu":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(steps)  # GPU: 50-step hipGraph replays
    if device != "cpu":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"device": device, "batch": batch, "steps": steps, "ms_per_step": 1e3 * dt / steps,
            "examples_per_sec": batch * steps / dt, "final_loss": tr.last_loss(),
            "hipgraph": getattr(tr, "graph_multi", None) is not None}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--steps", type=int, default=3000)
    a = ap.parse_args()
    for b in (32, 1024):
        print(json.dumps(run(a.device, b, a.steps if b == 32 else max(100, a.steps // 10), 20)), flush=True)
