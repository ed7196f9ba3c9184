"""Diagnostic: is one ResNet-50 fwd+bwd reproducible in one process? Same weights, same input, twice; with the
fused HIP BN/pool kernels and with them swapped for the PyTorch reference path."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mifx.models.resnet import resnet50_v2  # noqa: E402
import mifx.ops.bn_relu as bn  # noqa: E402
import mifx.models.resnet as rn  # noqa: E402


def run(batch, crop, native_bn=True, native_pool=True, amp=True, reps=3):
    torch.manual_seed(0)
    m = resnet50_v2(10).cuda().to(memory_format=torch.channels_last)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.rand(batch, 3, crop, crop, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (batch,), device="cuda", generator=g)
    old_ok, old_pool = bn.native_ok, rn.max_pool3s2
    if not native_bn:
        bn.native_ok = lambda t: False
    if not native_pool:
        rn.max_pool3s2 = lambda t: F.max_pool2d(t, 3, 2, 1)
    out = []
    try:
        for _ in range(reps):
            for p in m.parameters():
                p.grad = None
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                loss = F.cross_entropy(m(x).float(), y)
            loss.backward()
            torch.cuda.synchronize()
            out.append((float(loss), [p.grad.detach().float().clone() for p in m.parameters()]))
    finally:
        bn.native_ok, rn.max_pool3s2 = old_ok, old_pool
    l0, g0 = out[0]
    worst = 0.0
    for l, gg in out[1:]:
        for a, b in zip(gg, g0):
            worst = max(worst, ((a - b).norm() / (b.norm() + 1e-12)).item())
    print(f"batch {batch:3d} crop {crop:3d} bn={'hip' if native_bn else 'torch'} pool={'hip' if native_pool else 'torch'} "
          f"amp={amp}: losses {[round(l, 6) for l, _ in out]}  worst grad rel diff {worst:.3e}", flush=True)


if __name__ == "__main__":
    torch.backends.cudnn.benchmark = False
    for b, c in ((4, 64), (32, 224)):
        run(b, c)
        run(b, c, native_bn=False)
        run(b, c, native_bn=False, native_pool=False)
        run(b, c, amp=False)
    torch.backends.cudnn.deterministic = True
    print("cudnn.deterministic=True", flush=True)
    run(4, 64)
    run(4, 64, native_bn=False, native_pool=False)
