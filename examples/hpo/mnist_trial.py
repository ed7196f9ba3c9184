"""HPO worker: trains a small MNIST-shaped CNN with `--lr=`, `--num-layers=`, `--optimizer=` and prints
`Validation-accuracy=<v>` / `accuracy=<v>` for the metrics collector (the reference's worker runs
mxnet's train_mnist.py, `random-search-job.yaml:39-60`)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.data.synthetic import synthetic_images  # noqa: E402
from mifx.trainer.optim import make_optimizer  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--lr", type=float, default=0.02)
    ap.add_argument("--num-layers", type=int, default=2)
    ap.add_argument("--optimizer", default="sgd")
    ap.add_argument("--batch-size", type=int, default=64)
    ap.add_argument("--steps", type=int, default=150)
    a = ap.parse_args([x if not x.startswith("--") or "=" in x else x for x in (argv or sys.argv[1:])])
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    x, y = synthetic_images(4000, seed=5)
    x, y = x.flatten(1).to(dev), y.to(dev)
    layers, d = [], 784
    for _ in range(a.num_layers):
        layers += [nn.Linear(d, 128), nn.ReLU()]
        d = 128
    model = nn.Sequential(*layers, nn.Linear(d, 10)).to(dev)
    opt = make_optimizer(a.optimizer, model.parameters(), a.lr * (10 if a.optimizer == "ftrl" else 1))
    torch.manual_seed(0)
    for s in range(a.steps):
        idx = torch.randint(0, 3000, (a.batch_size,), device=dev)
        opt.zero_grad()
        F.cross_entropy(model(x[idx]), y[idx]).backward()
        opt.step()
    with torch.no_grad():
        acc = float((model(x[3000:]).argmax(1) == y[3000:]).float().mean())
    print(f"accuracy={acc:.4f}")
    print(f"Validation-accuracy={acc:.4f}")
    return acc


if __name__ == "__main__":
    main()
