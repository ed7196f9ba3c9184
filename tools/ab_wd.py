"""Interleaved A/B timing of fused W&D trainer variants in one process (removes box-to-box variance):
compact slab on/off x live weight staging on/off, at the throughput batch and the reference batch."""
import itertools
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    data = synthetic_records(1 << 22, device=dev, seed=1)
    res = {}
    for batch, steps in ((65536, 300), (40, 3000)):
        trs = {}
        for compact, live in itertools.product((False, True), (False, True)):
            tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device=dev, compact_slab=compact,
                                      live_staging=live)
            tr.set_data(data)
            tr.capture()
            trs[(compact, live)] = tr
        for _ in range(3):
            for key, tr in trs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    tr.step()
                torch.cuda.synchronize()
                us = 1e6 * (time.perf_counter() - t0) / steps
                res.setdefault(f"B={batch} compact={key[0]} live={key[1]}", []).append(round(us, 2))
    for k, v in res.items():
        print(json.dumps({"config": k, "us_per_step": v, "best": min(v)}), flush=True)


if __name__ == "__main__":
    main()
