"""Where do the fused and unfused channels_last ResNet-50 v2 passes diverge? Capture, per
BatchNormReLU2d, the forward input(s) and the gradient arriving at its output(s) in both runs and
print the relative difference layer by layer (forward order)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
import mifx.ops.bn_relu as bnr  # noqa: E402
from mifx.models.resnet import ResNetV2  # noqa: E402


def rel(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


def run(m, x, gout, native):
    rec = {}
    orig_f, orig_fa = bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add
    saved = bnr.native_ok

    def fwd(self, x):
        y = orig_f(self, x)
        e = rec.setdefault(self._nm, {})
        e["x"] = x.detach().clone()
        e["y"] = y.detach().clone()
        y.register_hook(lambda g: e.__setitem__("dy", g.detach().clone()))
        return y

    def fwd_add(self, a, b):
        y, s = orig_fa(self, a, b)
        e = rec.setdefault(self._nm, {})
        e["x"] = (a + b).detach().clone()
        e["y"] = y.detach().clone()
        y.register_hook(lambda g: e.__setitem__("dy", g.detach().clone()))
        s.register_hook(lambda g: e.__setitem__("ds", None if g is None else g.detach().clone()))
        a.register_hook(lambda g: e.__setitem__("da", g.detach().clone()))
        return y, s

    for n, mod in m.named_modules():
        if isinstance(mod, bnr.BatchNormReLU2d):
            mod._nm = n
    bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add = fwd, fwd_add
    if not native:
        bnr.native_ok = lambda t: False
    try:
        m.zero_grad()
        m(x).backward(gout)
    finally:
        bnr.BatchNormReLU2d.forward, bnr.BatchNormReLU2d.forward_add = orig_f, orig_fa
        bnr.native_ok = saved
    return rec


def main():
    torch.manual_seed(0)
    m = ResNetV2((1, 1, 1, 1), 10).cuda().to(memory_format=torch.channels_last)
    x = torch.rand(8, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
    gout = torch.randn(8, 10, device="cuda")
    ref = run(copy.deepcopy(m), x, gout, native=False)
    fus = run(copy.deepcopy(m), x, gout, native=True)
    for name in ref:
        r, f = ref[name], fus[name]
        parts = [f"{k} {rel(f[k], r[k]):.1e}" for k in ("x", "y", "dy", "ds", "da") if r.get(k) is not None and f.get(k) is not None]
        print(f"{name:16s} " + "  ".join(parts), flush=True)


if __name__ == "__main__":
    main()
