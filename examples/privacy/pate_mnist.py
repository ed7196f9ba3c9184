"""PATE end to end: partitioned teachers -> noisy-max labels for the student share -> student
training -> privacy analysis (reference: `research/pate_2017/train_teachers.py`,
`train_student.py`, `aggregation.py`, `analysis.py`). Synthetic MNIST-shaped data."""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.data.synthetic import synthetic_images
from mifx.models.cnn import PateCNN
from mifx.privacy.pate import aggregation, analysis2017


def partition_dataset(data, labels, nb_teachers: int, teacher_id: int):
    """Disjoint contiguous shard `teacher_id` of `nb_teachers` (reference `input.py:397-424`)."""
    n = len(data) // nb_teachers
    return data[teacher_id * n:(teacher_id + 1) * n], labels[teacher_id * n:(teacher_id + 1) * n]


def train(model, x, y, steps: int, batch: int, lr: float, dev):
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9)
    sched = torch.optim.lr_scheduler.ExponentialLR(opt, 0.1 ** (1.0 / max(1, steps)))
    model.train()
    for s in range(steps):
        idx = torch.randint(0, len(x), (batch,), device=dev)
        opt.zero_grad()
        F.cross_entropy(model(x[idx]), y[idx]).backward()
        opt.step()
        sched.step()
    model.eval()
    return model


@torch.no_grad()
def softmax_preds(model, x, batch: int = 4096):
    return torch.cat([F.softmax(model(x[i:i + batch]), -1) for i in range(0, len(x), batch)]).cpu().numpy()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--nb_teachers", type=int, default=10)
    ap.add_argument("--teacher_steps", type=int, default=300)
    ap.add_argument("--student_steps", type=int, default=300)
    ap.add_argument("--stdnt_share", type=int, default=1000)
    ap.add_argument("--lap_scale", type=float, default=10.0)
    ap.add_argument("--train_size", type=int, default=20000)
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args(argv)
    dev = torch.device(a.device)
    x, y = synthetic_images(a.train_size + 5000, seed=3)
    xtr, ytr = x[:a.train_size].to(dev), y[:a.train_size].to(dev)
    xte, yte = x[a.train_size:].to(dev), y[a.train_size:]
    preds = []
    for t in range(a.nb_teachers):
        torch.manual_seed(t)
        dx, dy = partition_dataset(xtr, ytr, a.nb_teachers, t)
        m = train(PateCNN().to(dev), dx, dy, a.teacher_steps, 128, 0.05, dev)
        preds.append(softmax_preds(m, xte[:a.stdnt_share]))
        print(f"teacher {t}: accuracy {aggregation.accuracy(preds[-1], yte[:a.stdnt_share].numpy()):.3f}")
    teachers = np.stack(preds)  # [T, N, C]
    stdnt_labels, clean_votes, _ = aggregation.noisy_max(teachers, a.lap_scale, return_clean_votes=True, seed=7,
                                                         device=dev if dev.type == "cuda" else None)
    print(f"aggregated label accuracy {aggregation.accuracy(stdnt_labels, yte[:a.stdnt_share].numpy()):.3f}")
    torch.manual_seed(99)
    student = train(PateCNN().to(dev), xte[:a.stdnt_share], torch.as_tensor(stdnt_labels, device=dev).long(),
                    a.student_steps, 128, 0.05, dev)
    acc = aggregation.accuracy(softmax_preds(student, xte[a.stdnt_share:]), yte[a.stdnt_share:].numpy())
    rep = analysis2017.analyze(clean_votes, noise_eps=1.0 / a.lap_scale, delta=1e-5, max_examples=a.stdnt_share)
    print(f"student accuracy {acc:.3f}; data-dependent eps {rep['eps']:.3f} "
          f"(data-independent {rep['data_independent_eps']:.3f})")
    return acc, rep


if __name__ == "__main__":
    main()
