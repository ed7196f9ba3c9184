"""Every convolution of ResNet-50 v2 at the training shape (B=256, 224x224, bf16 channels-last): the hand-written
kernels of csrc/gconv.hip against MIOpen, per pass -- forward, input gradient (stride 1: the forward kernel on dy
with the flipped weight; strided: the phase-split kernel), weight gradient (pixel-split kernel) -- called directly
(no autograd, no routing policy), CUDA-event timed. One JSON line per distinct shape with its count in the network
and the faster backend per pass; a last line sums the per-step time of all-MIOpen, all-HIP and best-per-pass.

    python tools/bench_resnet_convs.py > profiles/resnet_conv_routes_r4.jsonl
"""
import json
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.models.resnet import resnet50_v2  # noqa: E402
from mifx.ops import gconv  # noqa: E402


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def conv_shapes(batch=256, size=224):
    """(Hi, Wi, C, K, R, stride, pad) -> count, from a forward of the model with hooks (CPU, batch 1)."""
    m = resnet50_v2(1000)
    seen = Counter()

    def hook(mod, inp, out):
        x = inp[0]
        seen[(x.shape[2], x.shape[3], mod.in_channels, mod.out_channels, mod.kernel_size[0], mod.stride[0],
              mod.padding[0])] += 1

    for mod in m.modules():
        if isinstance(mod, nn.Conv2d):
            mod.register_forward_hook(hook)
    with torch.no_grad():
        m(torch.zeros(1, 3, size, size))
    return seen


def main():
    torch.backends.cudnn.benchmark = True
    B = int(os.environ.get("BATCH", "256"))
    tot = {"miopen": 0.0, "hip": 0.0, "best": 0.0}
    for (Hi, Wi, C, K, R, st, pad), cnt in sorted(conv_shapes().items()):
        rec = {"Hi": Hi, "C": C, "K": K, "R": R, "stride": st, "pad": pad, "count": cnt, "B": B}
        x = torch.randn(B, C, Hi, Wi, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (0.05 * torch.randn(K, C, R, R, device="cuda")).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        Ho, Wo = (Hi + 2 * pad - R) // st + 1, (Wi + 2 * pad - R) // st + 1
        dy = torch.randn(B, K, Ho, Wo, device="cuda", dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        hip_ok = gconv.eligible(x, w, 1, pad, st)
        t = {}
        t["fwd_miopen"] = timeit(lambda: F.conv2d(x, w, None, stride=st, padding=pad))
        # MIOpen through aten.convolution_backward, the op autograd runs (torch.nn.grad.conv2d_input / _weight take
        # a slower path on channels-last bf16)
        def mbwd(dg, wg):
            return torch.ops.aten.convolution_backward(dy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                       [dg, wg, False])

        t["dgrad_miopen"] = timeit(lambda: mbwd(True, False))
        t["wgrad_miopen"] = timeit(lambda: mbwd(False, True))
        t["bwd_both_miopen"] = timeit(lambda: mbwd(True, True))
        if hip_ok:
            w_fwd = w.view(1, K, C, R, R).permute(0, 1, 3, 4, 2).contiguous()
            t["fwd_hip"] = timeit(lambda: gconv._launch(x, w_fwd, None, B, Hi, Wi, 1, C, K, R, R, pad, False, st))
            if st == 1 and R - 1 - pad >= 0 and K % 32 == 0:
                w_bwd = w.view(1, K, C, R, R).flip(3, 4).permute(0, 2, 3, 4, 1).contiguous()
                t["dgrad_hip"] = timeit(lambda: gconv._launch(dy, w_bwd, None, B, Ho, Wo, 1, K, C, R, R, R - 1 - pad))
            elif st > 1:
                t["dgrad_hip"] = timeit(lambda: gconv.dgrad_strided(dy, w, B, Hi, Wi, 1, C, K, R, R, pad, st))
            if C % 8 == 0 and K % 8 == 0:
                t["wgrad_hip"] = timeit(lambda: gconv.wgrad(x, dy, B, Hi, Wi, 1, C, K, R, R, pad, st))
        best = {}
        for p in ("fwd", "dgrad", "wgrad"):
            h, mo = t.get(f"{p}_hip"), t[f"{p}_miopen"]
            best[p] = "hip" if h is not None and h < mo else "miopen"
            tot["miopen"] += cnt * mo
            tot["hip"] += cnt * (h if h is not None else mo)
            tot["best"] += cnt * min(mo, h if h is not None else mo)
        rec.update({k: round(v, 4) for k, v in t.items()})
        rec["route"] = best
        print(json.dumps(rec), flush=True)
    print(json.dumps({"summary_ms_per_step": {k: round(v, 3) for k, v in tot.items()}, "B": B}), flush=True)


if __name__ == "__main__":
    main()
