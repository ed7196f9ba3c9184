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


def train_all_teachers(a, nb_teachers: int, teacher_ids=None) -> list[float]:
    """Every teacher (or `teacher_ids`) in ONE grouped-network training run (`ensemble.train_ensemble`): same
    shards, batches, optimizer and checkpoint files as `train_teacher` per id. Under a multi-process launch
    (WORLD_SIZE > 1) rank r takes teachers r, r + WORLD_SIZE, ... (no communication)."""
    from . import ensemble

    os.makedirs(a.data_dir, exist_ok=True)
    os.makedirs(a.train_dir, exist_ok=True)
    if teacher_ids is None:
        rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
        teacher_ids = list(range(rank, nb_teachers, world))
        if world > 1 and (a.device is None or a.device == "cuda"):
            import torch

            if torch.cuda.is_available():
                a.device = f"cuda:{int(os.environ.get('LOCAL_RANK', rank)) % torch.cuda.device_count()}"
    if not teacher_ids:
        return []
    xtr, ytr, xte, yte = deep_cnn.load_dataset(a.dataset, train_size=a.train_size, test_size=a.test_size)
    shards = [deep_cnn.partition_dataset(xtr, ytr, nb_teachers, t) for t in teacher_ids]
    print(f"Training {len(teacher_ids)} teachers together; length of training data per teacher: {len(shards[0][1])}")
    cfg = config_from(a, nb_teachers)
    ckpts = [teacher_ckpt(a.train_dir, a.dataset, nb_teachers, t, a.deeper) for t in teacher_ids]
    assert ensemble.train_ensemble([s[0] for s in shards], [s[1] for s in shards], ckpts, cfg, device=a.device)
    preds = ensemble.ensemble_softmax_preds(xte, [f"{c}-{a.max_steps - 1}" for c in ckpts], cfg, device=a.device)
    precisions = [accuracy(p, yte) for p in preds]
    for t, p in zip(teacher_ids, precisions):
        print(f"Precision of teacher {t} after training: {p}")
    return precisions


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m mifx.privacy.pate.train_teachers")
    add_common_flags(ap)
    ap.add_argument("--nb_teachers", type=int, default=50)
    ap.add_argument("--teacher_id", type=int, default=0, help="-1: train every teacher at once (grouped ensemble)")
    a = ap.parse_args(argv)
    if a.teacher_id < 0:
        return train_all_teachers(a, a.nb_teachers)
    return train_teacher(a, a.nb_teachers, a.teacher_id)


if __name__ == "__main__":
    main()
