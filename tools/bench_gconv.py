"""Grouped conv microbench on the PATE ensemble's conv2 shape (G teachers x 64->128, 5x5 SAME, 14x14, B=128):
hand-written MFMA implicit GEMM (csrc/gconv.hip) vs MIOpen (F.conv2d), forward and input gradient, bf16."""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.ops import gconv  # noqa: E402


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


SHAPES = {"pate": [(250, 128, 14, 64, 128, 5), (50, 128, 14, 64, 128, 5), (1, 128, 14, 64, 128, 5)],
          # ResNet-50 3x3 stride-1 convs at B=256 (config 5)
          "resnet": [(1, 256, 56, 64, 64, 3), (1, 256, 28, 128, 128, 3), (1, 256, 14, 256, 256, 3),
                     (1, 256, 7, 512, 512, 3)],
          # ResNet-50 1x1 convs (B=256): expand / reduce of each stage
          "resnet1x1": [(1, 256, 56, 64, 256, 1), (1, 256, 56, 256, 64, 1), (1, 256, 28, 512, 128, 1),
                        (1, 256, 14, 1024, 256, 1), (1, 256, 7, 2048, 512, 1)]}
which = sys.argv[1] if len(sys.argv) > 1 else "pate"
for G, B, H, C, K, R in SHAPES[which]:
    x = torch.randn(B, G * C, H, H, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = 0.05 * torch.randn(G * K, C, R, R, device="cuda")
    b = torch.randn(G * K, device="cuda")
    wb, bb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last), b.to(torch.bfloat16)
    flop = 2.0 * B * H * H * G * K * C * R * R
    t_k = timeit(lambda: gconv.conv2d(x, w, b, padding=R // 2, groups=G))
    t_m = timeit(lambda: F.conv2d(x, wb, bb, padding=R // 2, groups=G))
    xr = x.detach().requires_grad_()
    yk = gconv.conv2d(xr, w, b, padding=R // 2, groups=G)
    dy = torch.randn_like(yk)
    t_kb = timeit(lambda: torch.autograd.grad(yk, xr, dy, retain_graph=True))
    ym = F.conv2d(xr, wb, bb, padding=R // 2, groups=G)
    t_mb = timeit(lambda: torch.autograd.grad(ym, xr, dy, retain_graph=True))
    wr = w.detach().requires_grad_()
    yw = gconv.conv2d(x, wr, b, padding=R // 2, groups=G)
    t_kw = timeit(lambda: torch.autograd.grad(yw, wr, dy, retain_graph=True))
    wm = wb.detach().requires_grad_()
    ywm = F.conv2d(x, wm, bb, padding=R // 2, groups=G)
    t_mw = timeit(lambda: torch.autograd.grad(ywm, wm, dy, retain_graph=True))
    print(json.dumps({"G": G, "B": B, "HW": H, "C": C, "K": K, "R": R, "fwd_ms_hip": t_k, "fwd_ms_miopen": t_m,
                      "fwd_tflops_hip": flop / t_k / 1e9, "fwd_tflops_miopen": flop / t_m / 1e9,
                      "dgrad_ms_hip": t_kb, "dgrad_ms_miopen": t_mb, "wgrad_ms_hip": t_kw,
                      "wgrad_ms_miopen": t_mw}), flush=True)
