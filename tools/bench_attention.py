"""BERT-base attention fwd+bwd microbenchmark: the hand-written fused kernel (csrc/attention.hip) against the
SDPA backends (B=32, h=12, S=128, d=64, bf16, key-padding mask, dropout 0.1). The fused kernel takes the
projection output [B, S, 3, h, d] directly; SDPA gets [B, h, S, d] views (the transposes are not timed)."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel


def run(backend, B=32, H=12, S=128, D=64, mask=True, drop=0.1, iters=50):
    torch.manual_seed(0)
    q, k, v = (torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    am = None
    if mask:
        am = torch.zeros(B, 1, 1, S, device="cuda", dtype=torch.bfloat16)
        am[:, :, :, S - 8:] = torch.finfo(torch.bfloat16).min
    g = torch.randn(B, H, S, D, device="cuda", dtype=torch.bfloat16)

    def step():
        with sdpa_kernel([backend]):
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=am, dropout_p=drop)
        o.backward(g)

    try:
        for _ in range(5):
            step()
    except RuntimeError as e:
        return {"backend": str(backend), "error": str(e).splitlines()[0][:120]}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    return {"backend": str(backend), "mask": mask, "us_fwd_bwd": (time.perf_counter() - t0) / iters * 1e6}


def run_fused(B=32, H=12, S=128, D=64, mask=True, drop=0.1, iters=50):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from mifx.ops import fused_bert as fb

    torch.manual_seed(0)
    qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    kb = None
    if mask:
        kb = torch.zeros(B, S, device="cuda")
        kb[:, S - 8:] = -1e30
    rng = torch.tensor([1, 2], dtype=torch.int64, device="cuda")
    g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)

    def step():
        fb.attention(qkv, kb, D ** -0.5, drop, rng, 0).backward(g)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        step()
    torch.cuda.synchronize()
    return {"backend": "mifx fused (csrc/attention.hip)", "mask": mask, "us_fwd_bwd": (time.perf_counter() - t0) / iters * 1e6}


def _tflops(r, B, H, S, D):
    # fwd 2 GEMMs (4 B H S^2 D FLOP) + bwd 5 (S recompute, dP, dQ, dK, dV: 10 B H S^2 D)
    if "us_fwd_bwd" in r:
        r["tflops"] = round(14 * B * H * S * S * D / (r["us_fwd_bwd"] * 1e-6) / 1e12, 1)
    r.update(B=B, S=S, H=H)
    return r


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--seq", type=int, nargs="*", default=[128])
    ap.add_argument("--tokens", type=int, default=4096, help="batch = tokens // seq")
    ap.add_argument("--drop", type=float, nargs="*", default=[0.1])
    ap.add_argument("--sdpa", action="store_true", help="also time the SDPA backends")
    a = ap.parse_args()
    for S in a.seq:
        B = max(1, a.tokens // S)
        for drop in a.drop:
            for mask in (True, False):
                print(json.dumps(_tflops(run_fused(B=B, S=S, mask=mask, drop=drop), B, 12, S, 64) | {"drop": drop}),
                      flush=True)
            if a.sdpa:
                for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
                    print(json.dumps(_tflops(run(be, B=B, S=S, mask=True, drop=drop), B, 12, S, 64) | {"drop": drop}),
                          flush=True)
