"""Time the small-CNN workloads of the reference: DP-SGD MNIST tutorial step (B=256, 256 microbatches,
`mnist_dpsgd_tutorial.py`), its non-private SGD step, PATE-2017 teacher step (B=128, `deep_cnn.py`) and the
TPU-notebook Keras CNN step (B=1024, Adam). One JSON line per workload."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.data.synthetic import synthetic_images  # noqa: E402
from mifx.models import cnn  # noqa: E402
from mifx.ops import dpsgd_mnist  # noqa: E402
from mifx.privacy import DPGradientDescentOptimizer, sparse_softmax_ce  # noqa: E402


def _time(fn, steps, warmup, dev):
    for _ in range(warmup):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def bench_dpsgd(dev, steps, warmup, dp=True, B=256, M=256, fused=True):
    x, y = synthetic_images(B * 8, seed=1)
    x, y = x.to(dev), y.to(dev)
    torch.manual_seed(0)
    model = cnn.MnistDPCNN().to(dev)
    # sparse_softmax_ce lets the fused MNIST gradient kernel run on the GPU; a plain lambda forces vmap(grad)
    vloss = sparse_softmax_ce if fused else (lambda out, t: F.cross_entropy(out, t, reduction="none"))
    if dp:
        opt = DPGradientDescentOptimizer(1.0, 1.12, M, model.parameters(), 0.08, seed=1)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=0.08)
    it = [0]

    def step():
        i = it[0] % 8
        it[0] += 1
        xb, yb = x[i * B:(i + 1) * B], y[i * B:(i + 1) * B]
        if dp:
            opt.step(model, vloss, xb, yb)
        elif fused and dev.type == "cuda":  # non-private step on the per-example gradient kernel
            dpsgd_mnist.assign_mean_grads(model, xb, yb)
            opt.step()
        else:
            opt.zero_grad()
            F.cross_entropy(model(xb), yb).backward()
            opt.step()

    dt = _time(step, steps, warmup, dev)
    name = ("dpsgd_mnist" + ("" if fused else "_vmap")) if dp else ("sgd_mnist" + ("_fused" if fused else ""))
    return {"workload": name, "batch": B, "microbatches": M if dp else None,
            "ms_per_step": 1e3 * dt, "examples_per_sec": B / dt}


def bench_model(dev, steps, warmup, name, model, B, shape, channels=1, lr=1e-3):
    x, y = synthetic_images(B * 4, shape=shape, channels=channels, seed=2)
    x, y = x.to(dev), y.to(dev)
    model = model.to(dev)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    it = [0]

    def step():
        i = it[0] % 4
        it[0] += 1
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(model(x[i * B:(i + 1) * B]), y[i * B:(i + 1) * B]).backward()
        opt.step()

    dt = _time(step, steps, warmup, dev)
    return {"workload": name, "batch": B, "ms_per_step": 1e3 * dt, "examples_per_sec": B / dt}


class _Logits(torch.nn.Module):
    """FashionCNN trains on its logits (forward() returns the served softmax)."""

    def __init__(self, m):
        super().__init__()
        self.m = m

    def forward(self, x):
        return self.m.logits(x)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device(a.device)
    torch.manual_seed(0)
    jobs = {
        "dpsgd": lambda: bench_dpsgd(dev, a.steps, a.warmup, dp=True),
        "dpsgd_vmap": lambda: bench_dpsgd(dev, a.steps, a.warmup, dp=True, fused=False),
        "dpsgd_m32": lambda: bench_dpsgd(dev, a.steps, a.warmup, dp=True, M=32),
        "sgd": lambda: bench_dpsgd(dev, a.steps, a.warmup, dp=False, fused=False),
        "sgd_fused": lambda: bench_dpsgd(dev, a.steps, a.warmup, dp=False),
        "pate": lambda: bench_model(dev, a.steps, a.warmup, "pate_teacher", cnn.PateCNN(), 128, (28, 28)),
        "tpu": lambda: bench_model(dev, a.steps, a.warmup, "tpu_mnist_cnn", cnn.TpuMnistCNN(), 1024, (28, 28)),
        "fashion": lambda: bench_model(dev, a.steps, a.warmup, "fashion_cnn", _Logits(cnn.FashionCNN()), 256, (28, 28)),
    }
    for k, fn in jobs.items():
        if (a.only and k not in a.only.split(",")) or (dev.type == "cpu" and k == "dpsgd_vmap"):
            continue
        r = fn()
        r["small_conv"] = os.environ.get("MIFX_SMALL_CONV", "0") == "1"
        print(json.dumps(r), flush=True)
