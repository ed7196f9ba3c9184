"""Per-layer precision of the fused BN+ReLU backward on activations captured from a real ResNet-50 v2
pass: for every BatchNormReLU2d, replay its (input, output-grad) pair through (a) the fused HIP
kernels in fp32, (b) PyTorch F.batch_norm in fp32, and compare both with fp64."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import mifx.ops.bn_relu as bnr  # noqa: E402
from mifx.models.resnet import ResNetV2  # noqa: E402


def rel(a, b):
    return ((a.double() - b).norm() / (b.norm() + 1e-30)).item()


def ref_bwd(x, w, b, dy, dtype):
    x = x.detach().to(dtype).requires_grad_()
    w2, b2 = w.detach().to(dtype).requires_grad_(), b.detach().to(dtype).requires_grad_()
    y = F.relu(F.batch_norm(x, None, None, w2, b2, True, 0.1, 1e-5))
    y.backward(dy.to(dtype))
    return y.detach(), x.grad, w2.grad, b2.grad


def main():
    torch.manual_seed(0)
    m = ResNetV2((1, 1, 1, 1), 10).cuda().to(memory_format=torch.channels_last)
    rec = []
    orig_f, orig_fa = bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add

    def fwd(self, x):
        bnr_native = bnr.native_ok
        bnr.native_ok = lambda t: False
        try:
            y = orig_f(self, x)
        finally:
            bnr.native_ok = bnr_native
        ent = {"name": getattr(self, "_nm", "?"), "x": x.detach().clone(), "w": self.weight, "b": self.bias}
        y.register_hook(lambda g: ent.__setitem__("dy", g.detach().clone()))
        rec.append(ent)
        return y

    def fwd_add(self, a, b):
        s = a + b
        return fwd(self, s), s

    for n, mod in m.named_modules():
        if isinstance(mod, bnr.BatchNormReLU2d):
            mod._nm = n
    bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add = fwd, fwd_add
    x = torch.rand(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    m(x).backward(torch.randn(8, 10, device="cuda"))
    bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add = orig_f, orig_fa

    print(f"{'layer':18s} {'M':>6s} {'C':>5s} {'|mu|/sd':>8s} | dx fused  dx ref32 | dw fused  dw ref32 | db fused  db ref32")
    for e in rec:
        xx, dy = e["x"], e["dy"].contiguous(memory_format=torch.channels_last)
        M = xx.numel() // xx.shape[1]
        mu = xx.double().mean((0, 2, 3))
        sd = xx.double().std((0, 2, 3))
        ratio = (mu.abs() / (sd + 1e-12)).max().item()
        y64, dx64, dw64, db64 = ref_bwd(xx, e["w"], e["b"], dy, torch.float64)
        _, dx32, dw32, db32 = ref_bwd(xx, e["w"], e["b"], dy, torch.float32)
        xf = xx.detach().clone().requires_grad_()
        wf, bf = e["w"].detach().clone().requires_grad_(), e["b"].detach().clone().requires_grad_()
        yf = bnr.bn_relu(xf, wf, bf, None, None, True)
        yf.backward(dy)
        print(f"{e['name']:18s} {M:6d} {xx.shape[1]:5d} {ratio:8.2f} | {rel(xf.grad, dx64):.1e}  {rel(dx32, dx64):.1e} | "
              f"{rel(wf.grad, dw64):.1e}  {rel(dw32, dw64):.1e} | {rel(bf.grad, db64):.1e}  {rel(db32, db64):.1e}  "
              f"y {rel(yf.detach(), y64):.1e}", flush=True)


if __name__ == "__main__":
    main()
