"""Notebook privacy/TensorFlow_Privacy (reference `notebooks/privacy/TensorFlow_Privacy.ipynb`):

* cell 3 — RDP accountant over the notebook's hyper-parameters (N=600, batch 32, noise 1.12, 1 epoch,
  delta 1e-5) with the notebook's order list, printed in the cell's format;
* cells 5-6 — DP-SGD on the MNIST tutorial CNN with 32 microbatches of the 32-example batch (vectorised
  per-example gradients + the fused HIP clip/noise kernel on the GPU, `csrc/dp.hip`).

Synthetic MNIST-shaped data stands in for the dataset (no downloads)."""
from __future__ import annotations

import argparse
import math
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.privacy import rdp  # noqa: E402

ORDERS = [1.25, 1.5, 1.75, 2., 2.25, 2.5, 3., 3.5, 4., 4.5] + list(range(5, 64)) + [128, 256, 512]


def apply_dp_sgd_analysis(q: float, sigma: float, steps: int, orders, delta: float) -> tuple[float, float]:
    r = rdp.compute_rdp(q, sigma, steps, orders)
    eps, _, opt_order = rdp.get_privacy_spent(orders, r, target_delta=delta)
    print(f"DP-SGD with sampling rate = {100 * q:.3g}% and noise_multiplier = {sigma} iterated over {steps} steps "
          f"satisfies differential privacy with eps = {eps:.3g} and delta = {delta}.")
    print(f"The optimal RDP order is {opt_order}.")
    if opt_order in (max(orders), min(orders)):
        print("The privacy estimate is likely to be improved by expanding the set of orders.")
    return eps, opt_order


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=600)
    ap.add_argument("--batch_size", type=int, default=32)
    ap.add_argument("--noise_multiplier", type=float, default=1.12)
    ap.add_argument("--epochs", type=float, default=1)
    ap.add_argument("--delta", type=float, default=1e-5)
    ap.add_argument("--train", type=int, default=1, help="also run the DP-SGD training cells")
    a = ap.parse_args(argv)
    q = a.batch_size / a.N
    if q > 1:
        raise SystemExit("N must be larger than the batch size.")
    steps = int(math.ceil(a.epochs * a.N / a.batch_size))
    eps, order = apply_dp_sgd_analysis(q, a.noise_multiplier, steps, ORDERS, a.delta)
    out = {"eps": eps, "opt_order": float(order)}
    if a.train:
        sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "privacy")))
        import mnist_dpsgd

        out["train"] = mnist_dpsgd.main(["--batch_size", str(a.batch_size), "--microbatches", str(a.batch_size),
                                         "--noise_multiplier", str(a.noise_multiplier), "--epochs", "1",
                                         "--learning_rate", "0.08", "--l2_norm_clip", "1.0",
                                         "--train_size", str(a.N)])
    return out


if __name__ == "__main__":
    main()
