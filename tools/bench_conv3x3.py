"""ResNet-50's 3x3 convolutions at B = 256 (stages 2-4; stage 1's 64-channel ones are not eligible): the implicit-GEMM
kernels (csrc/gemm8.hip CV 1 / CV 2, mifx.ops.conv3x3) against MIOpen (aten.convolution / convolution_backward, the
ops autograd runs) per pass -- forward (per tile configuration), stride-1 input gradient, weight gradient (grouped
split-K launch, per token chunk). One JSON line per measurement; each kernel result is checked against MIOpen's first.

usage: python tools/bench_conv3x3.py [--batch 256] [--passes fwd,dgrad,wgrad]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mifx.ops import gemm as hg  # noqa: E402

# (input H, C, Cout, stride) of every eligible ResNet-50 v2 conv2, with its count per network
SHAPES = [(56, 64, 64, 1, 3), (56, 128, 128, 2, 1), (28, 128, 128, 1, 3), (28, 256, 256, 2, 1), (14, 256, 256, 1, 5),
          (14, 512, 512, 2, 1), (7, 512, 512, 1, 2)]


def timeit(fn, iters=20):
    for _ in range(5):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    passes = a.passes.split(",")
    for h, c, cout, stride, count in SHAPES:
        n = a.batch
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(n, c, h, h, device="cuda", generator=g).to(torch.bfloat16) \
            .contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, c, 3, 3, device="cuda", generator=g) * (9 * c) ** -0.5) \
            .contiguous(memory_format=torch.channels_last)
        wb = w.to(torch.bfloat16)
        oh = (h - 1) // stride + 1
        M = n * oh * oh
        flop = 2.0 * M * cout * 9 * c
        tag = {"H": h, "C": c, "Cout": cout, "stride": stride, "count": count}
        w9 = wb.permute(0, 2, 3, 1).reshape(cout, 9 * c).contiguous()
        xn = x.permute(0, 2, 3, 1)
        if "fwd" in passes:
            ref = torch.ops.aten.convolution(x, wb, None, [stride] * 2, [1, 1], [1, 1], False, [0, 0], 1)
            us = timeit(lambda: torch.ops.aten.convolution(x, wb, None, [stride] * 2, [1, 1], [1, 1], False, [0, 0], 1))
            print(json.dumps({**tag, "pass": "fwd", "impl": "miopen", "us": round(us, 1),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)
            for cfg, (bm, bn) in enumerate(hg.gemm8_configs()):
                if M % bm or cout % bn:
                    continue
                y, _ = hg.gemm8_conv3x3(xn, w9, stride, 1, cfg=cfg)
                e = rel(y, ref.permute(0, 2, 3, 1).reshape(M, cout))
                us = timeit(lambda: hg.gemm8_conv3x3(xn, w9, stride, 1, cfg=cfg))
                print(json.dumps({**tag, "pass": "fwd", "impl": f"gemm8 {bm}x{bn}", "us": round(us, 1),
                                  "tflops": round(flop / us / 1e6, 1), "rel_err": round(e, 5)}), flush=True)
        dy = torch.randn(n, cout, oh, oh, device="cuda", generator=g).to(torch.bfloat16) \
            .contiguous(memory_format=torch.channels_last)
        if "dgrad" in passes and stride == 1:
            bw = lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [1, 1], [1, 1], [1, 1], False,  # noqa
                                                             [0, 0], 1, [True, False, False])[0]
            ref = bw()
            us = timeit(bw)
            print(json.dumps({**tag, "pass": "dgrad", "impl": "miopen", "us": round(us, 1),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)
            wt = w9.view(cout, 3, 3, c).flip(1, 2).permute(3, 1, 2, 0).reshape(c, 9 * cout).contiguous()
            dyn = dy.permute(0, 2, 3, 1)
            for cfg, (bm, bn) in enumerate(hg.gemm8_configs()):
                if M % bm or c % bn:
                    continue
                y, _ = hg.gemm8_conv3x3(dyn, wt, 1, 1, cfg=cfg)
                e = rel(y, ref.permute(0, 2, 3, 1).reshape(M, c))
                us = timeit(lambda: hg.gemm8_conv3x3(dyn, wt, 1, 1, cfg=cfg))
                print(json.dumps({**tag, "pass": "dgrad", "impl": f"gemm8 {bm}x{bn}", "us": round(us, 1),
                                  "tflops": round(flop / us / 1e6, 1), "rel_err": round(e, 5)}), flush=True)
        if "wgrad" in passes:
            bw = lambda: torch.ops.aten.convolution_backward(dy, x, wb, None, [stride] * 2, [1, 1], [1, 1], False,  # noqa
                                                             [0, 0], 1, [False, True, False])[1]
            ref = bw().float()
            us = timeit(bw)
            print(json.dumps({**tag, "pass": "wgrad", "impl": "miopen", "us": round(us, 1),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)
            geo = hg.conv_geo(n, h, h, c, stride, 1, x.device)
            dy2 = dy.permute(0, 2, 3, 1).reshape(M, cout)
            dw = torch.empty(cout, 3, 3, c, device="cuda")
            for chunk in ((2048, 4096, 8192, 16384) if c >= 128 and cout >= 128 else ()):  # (TN tiles >= 128)
                fn = lambda: hg.gemm8_tn_grouped([(dy2, xn, dw.view(cout, 9 * c), geo)], chunk=chunk,  # noqa
                                                 accumulate=False)
                fn()
                e = rel(dw.permute(0, 3, 1, 2), ref)
                us = timeit(fn)
                print(json.dumps({**tag, "pass": "wgrad", "impl": f"gemm8 grouped chunk {chunk}", "us": round(us, 1),
                                  "tflops": round(flop / us / 1e6, 1), "rel_err": round(e, 5)}), flush=True)
        del x, w, dy
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
