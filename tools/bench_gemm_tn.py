"""Weight-gradient GEMM dW = dY^T X on BERT-base's shapes (4096 tokens): the hand-written TN kernel
(csrc/gemm_tn.hip) at every configuration / split count against hipBLASLt (torch `dy.t() @ x`), with an accuracy check
against an fp32 reference. `python tools/bench_gemm_tn.py [--tokens 4096]` -> one JSON line per (shape, impl)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.ops import gemm  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            fn()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return 1e3 * st.elapsed_time(en) / (10 * reps)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=4096)
    a = ap.parse_args()
    T = a.tokens
    shapes = {"qkv": (2304, 768), "out": (768, 768), "ffn1": (3072, 768), "ffn2": (768, 3072)}
    torch.manual_seed(0)
    for name, (M, N) in shapes.items():
        dy = (torch.randn(T, M, device="cuda") * 0.5).to(torch.bfloat16)
        x = torch.randn(T, N, device="cuda").to(torch.bfloat16)
        ref = dy.float().t() @ x.float()
        fl = 2.0 * T * M * N
        us = timeit(lambda: dy.t() @ x)
        out = dy.t() @ x
        err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
        print(json.dumps({"gemm": name, "M": M, "N": N, "T": T, "impl": "hipblaslt dy.t() @ x", "us": round(us, 2),
                          "tflops": round(fl / us / 1e6, 1), "max_rel_err": round(err, 5)}), flush=True)
        pk = gemm.pick_tn(M, N, T)
        for cfg, (bm, bn, opt) in enumerate(gemm.tn_configs()):
            if M % bm or N % bn:
                continue
            for s in (1, 2, 4, 8):
                if T % (64 * s) or (M // bm) * (N // bn) * s > 1024 or (opt & 2):
                    continue
                out = gemm.gemm_tn(dy, x, cfg, s)
                err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                us = timeit(lambda: gemm.gemm_tn(dy, x, cfg, s))
                print(json.dumps({"gemm": name, "M": M, "N": N, "T": T, "impl": f"hip tn cfg{cfg} {bm}x{bn} opt{opt} "
                                  f"splits{s}", "picked": pk == (cfg, s), "us": round(us, 2),
                                  "tflops": round(fl / us / 1e6, 1), "max_rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
