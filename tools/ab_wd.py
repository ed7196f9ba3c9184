"""Interleaved A/B timing of fused W&D trainer variants in one process (removes box-to-box variance):
the register-chained kernel (csrc/wd_chain.hip) vs the LDS-tile kernel (csrc/wide_deep.hip), at several
throughput batches and the reference batch. `--kernels chain,tile --batches 65536,40`."""
import argparse
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="chain8,chain4,tile",
                    help="chain8 / chain4 (waves), tile, t64 (T = 64 build, batch <= 64), or chain8tail / chain8notail "
                         "(in-kernel step tail on / off)")
    ap.add_argument("--batches", default="65536,131072,40")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps-per-graph", type=int, default=10, help="as bench.py; 1 = launch-bound replays")
    a = ap.parse_args()
    dev = torch.device("cuda")
    data = synthetic_records(1 << 22, device=dev, seed=1)
    res = {}
    for batch in (int(b) for b in a.batches.split(",")):
        steps = 3000 if batch <= 1024 else 300
        trs = {}
        for k in a.kernels.split(","):
            if k == "tile":
                kw = {"kernel": "tile"}
            elif k == "t64":  # the T = 64 build (csrc/wd_chain64.hip), batches <= 64
                kw = {"kernel": "chain", "small_tile": True}
            else:
                tail = None if not k.endswith("tail") else (not k.endswith("notail"))
                kw = {"kernel": "chain", "waves": int(k[5:6] or 8), "in_kernel_tail": tail, "small_tile": False}
            tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device=dev, **kw)
            tr.set_data(data)
            tr.capture(steps_per_graph=a.steps_per_graph)
            trs[k] = tr
        for _ in range(a.rounds):
            for key, tr in trs.items():
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                tr.run(steps)
                torch.cuda.synchronize()
                us = 1e6 * (time.perf_counter() - t0) / steps
                res.setdefault(f"B={batch} kernel={key}", []).append(round(us, 2))
        for key, tr in trs.items():
            res.setdefault(f"B={batch} kernel={key} loss", []).append(round(tr.last_loss() / batch, 5))
        del trs
    for k, v in res.items():
        print(json.dumps({"config": k, "values": v, "best": min(v)}), flush=True)


if __name__ == "__main__":
    main()
