"""Stem max-pool (3x3 / s2 / p1, NHWC bf16) forward and backward at ResNet-50's B=256 shape: CUDA-event time per
call and the bytes each pass must move (x / dx 411 MB, y / dy 103 MB, 1-byte argmax 51 MB)."""
import hashlib
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.ops.pool import max_pool3s2  # noqa: E402


def main():
    N, C, H, W = 256, 64, 112, 112
    torch.manual_seed(0)
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x.requires_grad_()
    y = max_pool3s2(x)
    g = torch.randn_like(y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def t(fn, it=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(it):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / it

    dx = torch.autograd.grad(max_pool3s2(x), x, g)[0]
    ydig = hashlib.sha256(max_pool3s2(x.detach()).contiguous().view(torch.int16).cpu().numpy().tobytes())
    digest = hashlib.sha256(dx.contiguous(memory_format=torch.channels_last).view(torch.int16).cpu().numpy().tobytes())
    fwd = t(lambda: max_pool3s2(x.detach()))
    both = t(lambda: torch.autograd.grad(max_pool3s2(x), x, g))
    xb, yb = x.numel() * 2, y.numel() * 2
    print(json.dumps({"fwd_us": round(fwd, 1), "bwd_us": round(both - fwd, 1),
                      "fwd_TBps": round((xb + yb + yb / 2) / fwd / 1e6, 2),
                      "bwd_TBps": round((xb + yb + yb / 2) / (both - fwd) / 1e6, 2),
                      "y_sha256": ydig.hexdigest()[:16], "dx_sha256": digest.hexdigest()[:16],
                      "pair_fwd": os.environ.get("MIFX_POOL_PAIR", "1") != "0",
                      "even_bwd": os.environ.get("MIFX_POOL_EVEN", "1") != "0"}), flush=True)


if __name__ == "__main__":
    main()
