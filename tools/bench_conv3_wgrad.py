"""Per-shape time of the 3x3 weight gradient: the nine-tap kernel (mifx.ops.conv3_wgrad) vs MIOpen
(aten.convolution_backward, weight gradient only), ResNet-50's 64/128-channel shapes at B = 256. One JSON line per
(shape, impl) on stdout."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mifx.ops import conv3_wgrad

SHAPES = [(56, 64, 64, 1, 3), (28, 128, 128, 1, 3), (56, 128, 128, 2, 1)]  # (H, C, Cout, stride, count in the net)


def timed(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for h, c, cout, s, cnt in SHAPES:
        oh = (h - 1) // s + 1
        x = torch.randn(a.batch, c, h, h, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        dy = torch.randn(a.batch, cout, oh, oh, device=dev).bfloat16().contiguous(memory_format=torch.channels_last)
        w = torch.randn(cout, c, 3, 3, device=dev).contiguous(memory_format=torch.channels_last)
        wb = w.bfloat16()
        flops = 2.0 * a.batch * oh * oh * cout * 9 * c
        mine = conv3_wgrad.wgrad(x, dy, w, s)
        lib = torch.ops.aten.convolution_backward(dy, x, wb, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                  [False, True, False])[1].float()
        err = float((mine - lib).norm() / lib.norm())
        for impl, fn in (("hip nine-tap", lambda: conv3_wgrad.wgrad(x, dy, w, s)),
                         ("miopen", lambda: torch.ops.aten.convolution_backward(
                             dy, x, wb, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))):
            us = timed(fn, a.iters)
            print(json.dumps({"H": h, "C": c, "Cout": cout, "stride": s, "count": cnt, "pass": "wgrad", "impl": impl,
                              "us": round(us, 1), "tflops": round(flops / us / 1e6, 1), "rel_err_vs_miopen": err}),
                  flush=True)


if __name__ == "__main__":
    main()
