"""Is the fused-BN ResNet gradient mismatch a bug or conditioning? Compare, against an fp64 NCHW
reference: fp32 NCHW (F.batch_norm), fp32 channels_last with the BN kernels disabled (same MIOpen
NHWC convolutions, PyTorch BN), and fp32 channels_last with the fused HIP BN kernels."""
import copy
import sys

import torch

sys.path.insert(0, ".")
import mifx.ops.bn_relu as bnr  # noqa: E402
from mifx.models.resnet import ResNetV2  # noqa: E402


def grads(m, x, gout):
    m.zero_grad()
    out = m(x)
    out.backward(gout.to(out.dtype))
    return out.detach().double(), {n: p.grad.detach().double().clone() for n, p in m.named_parameters()}


def rel_fro(a, b):
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def main():
    native_ok = bnr.native_ok
    cases = [((1, 1, 1, 1), 64, 8, True), ((1, 1, 1, 1), 64, 8, False), ((3, 4, 6, 3), 64, 4, False)]
    for layers, hw, bs, tf32 in cases:
        torch.backends.cudnn.allow_tf32 = tf32
        torch.backends.cuda.matmul.allow_tf32 = tf32
        torch.manual_seed(0)
        m = ResNetV2(layers, 10).cuda()
        x = torch.rand(bs, 3, hw, hw, device="cuda")
        gout = torch.randn(bs, 10, device="cuda")
        o64, g64 = grads(copy.deepcopy(m).double(), x.double(), gout.double())
        o32, g32 = grads(copy.deepcopy(m), x, gout)
        xl = x.contiguous(memory_format=torch.channels_last)
        bnr.native_ok = lambda t: False
        try:
            ol, gl = grads(copy.deepcopy(m).to(memory_format=torch.channels_last), xl, gout)
        finally:
            bnr.native_ok = native_ok
        of, gf = grads(copy.deepcopy(m).to(memory_format=torch.channels_last), xl, gout)
        rows = [(rel_fro(gf[n], g64[n]), rel_fro(gl[n], g64[n]), rel_fro(g32[n], g64[n]), n) for n in g64]
        rows.sort(reverse=True)
        cat = lambda g: torch.cat([v.flatten() for v in g.values()])  # noqa: E731
        print(f"layers={layers} hw={hw} bs={bs} allow_tf32={tf32}: out err nchw32={(o32 - o64).abs().max().item():.2e} "
              f"nhwc32={(ol - o64).abs().max().item():.2e} fused={(of - o64).abs().max().item():.2e}")
        print(f"   global rel-fro: fused {rel_fro(cat(gf), cat(g64)):.2e}  nhwc32 {rel_fro(cat(gl), cat(g64)):.2e}  "
              f"nchw32 {rel_fro(cat(g32), cat(g64)):.2e}")
        ratio = max(r[0] / max(r[1], r[2], 1e-7) for r in rows)
        print(f"   max per-param ratio fused/max(ref32s) = {ratio:.2f}")
        for ef, el, e32, n in rows[:6]:
            print(f"   {n:36s} rel-fro fused {ef:.2e}  nhwc32 {el:.2e}  nchw32 {e32:.2e}", flush=True)


if __name__ == "__main__":
    main()
