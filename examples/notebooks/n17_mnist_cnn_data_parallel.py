"""Notebook tpu/Keras_MNIST_TPU re-targeted to MI355X data parallelism (reference
`notebooks/tpu/Keras_MNIST_TPU.ipynb` cells 11-26): CNN Conv32-Pool-Conv64-Pool-Conv64-Dense64-
Dropout-Dense10, global batch 1024 with drop_remainder, Adam 1e-3, fit(steps_per_epoch=60,
epochs=10), save_weights and "sync to CPU" for inference.

`keras_to_tpu_model(TPUDistributionStrategy)` becomes one process per GPU: launch with
`python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ...`; the global batch
is split over the ranks, gradients are all-reduced in buckets over RCCL (gloo on CPU) by
mifx.parallel.DataParallel, and rank 0 writes the weights (safetensors). Synthetic MNIST-shaped data."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from safetensors.torch import load_file, save_file  # noqa: E402

from mifx.data.synthetic import synthetic_images  # noqa: E402
from mifx.models.cnn import TpuMnistCNN  # noqa: E402
from mifx.parallel import dist as mdist  # noqa: E402
from mifx.parallel.ddp import DataParallel  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch_size", type=int, default=1024, help="global batch (split over ranks)")
    ap.add_argument("--steps_per_epoch", type=int, default=60)
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--train_size", type=int, default=60000)
    ap.add_argument("--weights", default=os.path.join(tempfile.gettempdir(), "mnist_cnn.safetensors"))
    a = ap.parse_args(argv)
    env = mdist.init()
    dev = torch.device("cuda", env.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    per_rank = a.batch_size // env.world_size
    x, y = synthetic_images(a.train_size + 2000, seed=11)
    x = x.unsqueeze(1)
    xtr, ytr = x[:a.train_size].to(dev), y[:a.train_size].to(dev)
    xte, yte = x[a.train_size:], y[a.train_size:]
    torch.manual_seed(0)
    model = TpuMnistCNN().to(dev)
    if dev.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    dp = DataParallel(model)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    nb = a.train_size // a.batch_size  # drop_remainder=True
    g = torch.Generator(device="cpu").manual_seed(1234)
    t0 = time.perf_counter()
    for ep in range(a.epochs):
        perm = torch.randperm(a.train_size, generator=g).to(dev)  # same shuffle on every rank
        tot = 0.0
        for s in range(a.steps_per_epoch):
            b = s % nb
            idx = perm[b * a.batch_size + env.rank * per_rank: b * a.batch_size + (env.rank + 1) * per_rank]
            opt.zero_grad(set_to_none=True)
            with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
                logits = dp(xtr[idx])
            loss = F.cross_entropy(logits.float(), ytr[idx])
            loss.backward()
            dp.finish()
            opt.step()
            tot += float(loss.detach())
        if env.is_main:
            print(f"Epoch {ep + 1}/{a.epochs} - loss: {tot / a.steps_per_epoch:.4f}")
    if dev.type == "cuda":
        torch.cuda.synchronize()
    secs = time.perf_counter() - t0
    ex_per_s = a.epochs * a.steps_per_epoch * a.batch_size / secs
    res = {"examples_per_sec": ex_per_s, "world_size": env.world_size}
    if env.is_main:
        save_file({k: v.detach().cpu().contiguous() for k, v in model.state_dict().items()}, a.weights)
        cpu_model = TpuMnistCNN()                                   # sync_to_cpu: inference on host
        cpu_model.load_state_dict(load_file(a.weights))
        cpu_model.eval()
        with torch.no_grad():
            res["test_accuracy"] = float((cpu_model(xte).argmax(1) == yte).float().mean())
        print(f"examples/sec {ex_per_s:.0f} on {env.world_size} rank(s); test accuracy {res['test_accuracy']:.4f}")
    mdist.shutdown()
    return res


if __name__ == "__main__":
    main()
