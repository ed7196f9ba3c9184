"""Train one teacher of a PATE ensemble on its disjoint data shard (reference
`research/pate_2017/train_teachers.py:28-96`; flags and checkpoint naming kept:
`<train_dir>/<dataset>_<nb>_teachers_<id>[_deep].ckpt-<max_steps-1>`).

    python -m mifx.privacy.pate.train_teachers --dataset mnist --nb_teachers 10 --teacher_id 0"""
from __future__ import annotations

import argparse
import os

from . import deep_cnn
from .aggregation import accuracy


def teacher_ckpt(train_dir: str, dataset: str, nb_teachers: int, teacher_id: int, deeper: bool) -> str:
    name = f"{nb_teachers}_teachers_{teacher_id}{'_deep' if deeper else ''}.ckpt"
    return os.path.join(train_dir, f"{dataset}_{name}")


def add_common_flags(ap: argparse.ArgumentParser) -> None:
    ap.add_argument("--dataset", default="svhn")
    ap.add_argument("--nb_labels", type=int, default=10)
    ap.add_argument("--data_dir", default="/tmp")
    ap.add_argument("--train_dir", default="/tmp/train_dir")
    ap.add_argument("--max_steps", type=int, default=3000)
    ap.add_argument("--deeper", action="store_true")
    ap.add_argument("--batch_size", type=int, default=128)
    ap.add_argument("--learning_rate", type=int, default=5)
    ap.add_argument("--epochs_per_decay", type=int, default=350)
    ap.add_argument("--train_size", type=int, default=None, help="synthetic train rows (default: dataset size)")
    ap.add_argument("--test_size", type=int, default=None)
    ap.add_argument("--device", default=None)


def config_from(a, nb_teachers: int) -> deep_cnn.DeepCNNConfig:
    return deep_cnn.DeepCNNConfig(dataset=a.dataset, nb_labels=a.nb_labels, batch_size=a.batch_size,
                                  epochs_per_decay=a.epochs_per_decay, learning_rate=a.learning_rate,
                                  max_steps=a.max_steps, nb_teachers=nb_teachers, deeper=a.deeper)


def train_teacher(a, nb_teachers: int, teacher_id: int) -> float:
    os.makedirs(a.data_dir, exist_ok=True)
    os.makedirs(a.train_dir, exist_ok=True)
    xtr, ytr, xte, yte = deep_cnn.load_dataset(a.dataset, train_size=a.train_size, test_size=a.test_size)
    data, labels = deep_cnn.partition_dataset(xtr, ytr, nb_teachers, teacher_id)
    print("Length of training data: " + str(len(labels)))
    cfg = config_from(a, nb_teachers)
    ckpt = teacher_ckpt(a.train_dir, a.dataset, nb_teachers, teacher_id, a.deeper)
    assert deep_cnn.train(data, labels, ckpt, cfg, device=a.device)
    preds = deep_cnn.softmax_preds(xte, f"{ckpt}-{a.max_steps - 1}", cfg, device=a.device)
    precision = accuracy(preds, yte)
    print("Precision of teacher after training: " + str(precision))
    return precision


def main(argv=None) -> float:
    ap = argparse.ArgumentParser(prog="python -m mifx.privacy.pate.train_teachers")
    add_common_flags(ap)
    ap.add_argument("--nb_teachers", type=int, default=50)
    ap.add_argument("--teacher_id", type=int, default=0)
    a = ap.parse_args(argv)
    return train_teacher(a, a.nb_teachers, a.teacher_id)


if __name__ == "__main__":
    main()
