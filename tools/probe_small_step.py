"""Where the reference-batch W&D step goes: hipGraphs of 10 x {fused + optimizer}, 10 x fused alone, 10 x optimizer
alone, 10 x {fused + a trivial kernel}, timed by replays (us per step). `python tools/probe_small_step.py [--batch 40]`"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.ops import wide_deep as wdk  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=40)
    ap.add_argument("--reps", type=int, default=300)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    for small in (True, False):
        tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=a.batch, device=dev, small_tile=small)
        tr.set_data(synthetic_records(1 << 16, device=dev, seed=3))
        tiny = torch.zeros(64, device=dev)

        def fused():
            tr._launch(tr.records, tr.n_data, tr.batch, 0, tr.step_ctr, tr.slab, tr.slab_loss, None, tr.grid, True)

        def opt():
            tr._apply()

        def triv():
            tiny.add_(1.0)

        variants = {"fused+opt": (fused, opt), "fused": (fused,), "opt": (opt,), "fused+trivial": (fused, triv),
                    "trivial": (triv,)}
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            for fns in variants.values():
                for f in fns:
                    f()
        torch.cuda.current_stream(dev).wait_stream(s)
        graphs = {}
        for name, fns in variants.items():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(10):
                    for f in fns:
                        f()
            graphs[name] = g
        for _ in range(3):
            for name, g in graphs.items():
                g.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.reps):
                    g.replay()
                torch.cuda.synchronize()
                us = 1e6 * (time.perf_counter() - t0) / (10 * a.reps)
                key = f"tile={tr.tile} {name}"
                res[key] = min(res.get(key, 1e9), us)
        del tr, graphs
    for k, v in res.items():
        print(json.dumps({"batch": a.batch, "variant": k, "us_per_step": round(v, 2)}), flush=True)


if __name__ == "__main__":
    main()
