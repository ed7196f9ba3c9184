"""MIOpen time of the ResNet-50 convolutions that stay off the implicit-GEMM kernels at B = 256 (stage 1's 64-channel
convolutions, the stride-2 1x1 shortcuts, the stem), per pass, through the ops autograd runs (aten.convolution /
convolution_backward). One JSON line per (conv, pass)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (name, H, C, K, R, stride, pad, count per step)
CONVS = [("s1_3x3_64", 56, 64, 64, 3, 1, 1, 3), ("s1_conv1_64_64", 56, 64, 64, 1, 1, 0, 1),
         ("s1_conv1_256_64", 56, 256, 64, 1, 1, 0, 2), ("s1_conv3_64_256", 56, 64, 256, 1, 1, 0, 3),
         ("s1_shortcut_64_256", 56, 64, 256, 1, 1, 0, 1), ("s2_shortcut", 56, 256, 512, 1, 2, 0, 1),
         ("s3_shortcut", 28, 512, 1024, 1, 2, 0, 1), ("s4_shortcut", 14, 1024, 2048, 1, 2, 0, 1),
         ("stem", 224, 3, 64, 7, 2, 3, 1)]


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


def main():
    torch.backends.cudnn.benchmark = True
    n = 256
    tot = 0.0
    for name, h, c, k, r, s, p, count in CONVS:
        x = torch.randn(n, c, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(k, c, r, r, device="cuda") * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.ops.aten.convolution(x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1)
        dy = torch.randn_like(y)
        res = {"conv": name, "count": count}
        res["fwd_us"] = timeit(lambda: torch.ops.aten.convolution(x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1))
        res["dgrad_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]))
        res["wgrad_us"] = timeit(lambda: torch.ops.aten.convolution_backward(
            dy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [False, True, False]))
        res["per_step_us"] = round(count * (res["fwd_us"] + res["dgrad_us"] + res["wgrad_us"]), 1)
        tot += res["per_step_us"]
        print(json.dumps({kk: (round(v, 1) if isinstance(v, float) else v) for kk, v in res.items()}), flush=True)
        del x, w, y, dy
        torch.cuda.empty_cache()
    print(json.dumps({"total_per_step_us": round(tot, 1)}), flush=True)


if __name__ == "__main__":
    main()
