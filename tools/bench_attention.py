"""BERT-base attention fwd+bwd microbenchmark across SDPA backends (B=32, h=12, S=128, d=64, bf16,
key-padding mask, dropout 0.1) -> which backend the BERT layer should use on MI355X."""
import json
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


if __name__ == "__main__":
    for be in (SDPBackend.FLASH_ATTENTION, SDPBackend.EFFICIENT_ATTENTION, SDPBackend.MATH):
        for mask in (True, False):
            print(json.dumps(run(be, mask=mask)), flush=True)
