"""DP-SGD on the MNIST tutorial CNN (reference: `notebooks/privacy/privacy/tutorials/mnist_dpsgd_tutorial.py`).

Flags mirror the tutorial (lr 0.08, noise 1.12, clip 1.0, batch 256, microbatches 256, epochs 60);
synthetic MNIST-shaped data stands in for the dataset (no downloads). Prints per-epoch test accuracy
and the epsilon spent (RDP accountant, delta 1e-5)."""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.data.synthetic import synthetic_images
from mifx.models.cnn import MnistDPCNN
from mifx.ops import dpsgd_mnist
from mifx.privacy import DPGradientDescentOptimizer, compute_dp_sgd_privacy, sparse_softmax_ce


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--dpsgd", type=int, default=1)
    ap.add_argument("--learning_rate", type=float, default=0.08)
    ap.add_argument("--noise_multiplier", type=float, default=1.12)
    ap.add_argument("--l2_norm_clip", type=float, default=1.0)
    ap.add_argument("--batch_size", type=int, default=256)
    ap.add_argument("--microbatches", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=60)
    ap.add_argument("--train_size", type=int, default=60000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args(argv)
    if a.batch_size % a.microbatches:
        raise ValueError("Number of microbatches should divide evenly batch_size")
    dev = torch.device(a.device)
    x, y = synthetic_images(a.train_size + 10000, seed=1)
    xtr, ytr, xte, yte = x[:a.train_size].to(dev), y[:a.train_size].to(dev), x[a.train_size:].to(dev), \
        y[a.train_size:].to(dev)
    torch.manual_seed(0)
    model = MnistDPCNN().to(dev)
    vloss = sparse_softmax_ce  # per-example loss; lets the fused MNIST gradient kernel run on the GPU
    if a.dpsgd:
        opt = DPGradientDescentOptimizer(a.l2_norm_clip, a.noise_multiplier, a.microbatches, model.parameters(),
                                         a.learning_rate, seed=1234)
    else:
        opt = torch.optim.SGD(model.parameters(), lr=a.learning_rate)
    steps_per_epoch = a.train_size // a.batch_size
    fused_plain = not a.dpsgd and dpsgd_mnist.supported(model, xtr)
    for epoch in range(1, a.epochs + 1):
        t0 = time.time()
        perm = torch.randperm(a.train_size, device=dev)
        for s in range(steps_per_epoch):
            idx = perm[s * a.batch_size:(s + 1) * a.batch_size]
            if a.dpsgd:
                opt.step(model, vloss, xtr[idx], ytr[idx])
            elif fused_plain:  # same network, non-private: per-example gradient kernel + mean (csrc/dpsgd_mnist.hip)
                dpsgd_mnist.assign_mean_grads(model, xtr[idx], ytr[idx])
                opt.step()
            else:
                opt.zero_grad()
                F.cross_entropy(model(xtr[idx]), ytr[idx]).backward()
                opt.step()
        with torch.no_grad():
            acc = float((model(xte).argmax(1) == yte).float().mean())
        msg = f"epoch {epoch}: test accuracy {acc:.4f} ({(time.time() - t0):.1f}s)"
        if a.dpsgd:
            eps, _ = compute_dp_sgd_privacy(a.train_size, a.batch_size, a.noise_multiplier, epoch, 1e-5)
            msg += f"; eps = {eps:.2f} for delta=1e-5"
        print(msg, flush=True)
    return acc


if __name__ == "__main__":
    main()
