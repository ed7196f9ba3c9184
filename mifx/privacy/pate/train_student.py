"""Train a PATE student on teacher-ensemble labels aggregated with Laplace noisy-max (reference
`research/pate_2017/train_student.py:32-200`): ensemble softmax predictions on the first
`stdnt_share` test images -> noisy_max (HIP Philox/Laplace kernel on the GPU) -> student training
-> accuracy on the remaining test images. `--save_labels` dumps clean votes / teacher labels /
student labels as .npy under data_dir with the reference file names.

    python -m mifx.privacy.pate.train_student --dataset mnist --nb_teachers 10 --stdnt_share 1000"""
from __future__ import annotations

import argparse
import os

import numpy as np

from . import aggregation, deep_cnn
from .train_teachers import add_common_flags, config_from, teacher_ckpt


def ensemble_preds(a, nb_teachers: int, stdnt_data: np.ndarray, chunk: int = 64) -> np.ndarray:
    """[nb_teachers, N, labels] teacher softmax predictions; `chunk` teachers per grouped forward
    (`ensemble.ensemble_softmax_preds`) instead of one restore + inference per teacher."""
    from .ensemble import ensemble_softmax_preds

    out = np.zeros((nb_teachers, len(stdnt_data), a.nb_labels), dtype=np.float32)
    cfg = config_from(a, nb_teachers)
    ckpts = [teacher_ckpt(a.teachers_dir, a.dataset, nb_teachers, t, a.deeper) + f"-{a.teachers_max_steps - 1}"
             for t in range(nb_teachers)]
    for t0 in range(0, nb_teachers, chunk):
        out[t0:t0 + chunk] = ensemble_softmax_preds(stdnt_data, ckpts[t0:t0 + chunk], cfg, device=a.device)
        print(f"Computed Teachers {t0}..{min(nb_teachers, t0 + chunk) - 1} softmax predictions")
    return out


def prepare_student_data(a, nb_teachers: int, save: bool = False):
    os.makedirs(a.train_dir, exist_ok=True)
    _, _, test_data, test_labels = deep_cnn.load_dataset(a.dataset, train_size=a.train_size, test_size=a.test_size)
    assert a.stdnt_share < len(test_data)
    stdnt_data = test_data[:a.stdnt_share]
    teachers_preds = ensemble_preds(a, nb_teachers, stdnt_data)
    dev = a.device
    if dev is None:
        import torch

        dev = "cuda" if torch.cuda.is_available() else None
    if not save:
        stdnt_labels = aggregation.noisy_max(teachers_preds, a.lap_scale, device=dev)
    else:
        stdnt_labels, clean_votes, labels_for_dump = aggregation.noisy_max(teachers_preds, a.lap_scale,
                                                                           return_clean_votes=True, device=dev)
        base = os.path.join(a.data_dir, f"{a.dataset}_{nb_teachers}")
        np.save(f"{base}_student_clean_votes_lap_{a.lap_scale}.npy", clean_votes)
        np.save(f"{base}_teachers_labels_lap_{a.lap_scale}.npy", labels_for_dump)
        np.save(f"{base}_student_labels_lap_{a.lap_scale}.npy", stdnt_labels)
    print("Accuracy of the aggregated labels: " + str(aggregation.accuracy(stdnt_labels, test_labels[:a.stdnt_share])))
    return stdnt_data, np.asarray(stdnt_labels, np.int32), test_data[a.stdnt_share:], test_labels[a.stdnt_share:]


def train_student(a, nb_teachers: int) -> float:
    stdnt_data, stdnt_labels, test_data, test_labels = prepare_student_data(a, nb_teachers, save=a.save_labels)
    name = f"{a.dataset}_{nb_teachers}_student{'_deeper' if a.deeper else ''}.ckpt"
    ckpt = os.path.join(a.train_dir, name)
    cfg = config_from(a, nb_teachers)
    assert deep_cnn.train(stdnt_data, stdnt_labels, ckpt, cfg, device=a.device)
    preds = deep_cnn.softmax_preds(test_data, f"{ckpt}-{a.max_steps - 1}", cfg, device=a.device)
    precision = aggregation.accuracy(preds, test_labels)
    print("Precision of student after training: " + str(precision))
    return precision


def main(argv=None) -> float:
    ap = argparse.ArgumentParser(prog="python -m mifx.privacy.pate.train_student")
    add_common_flags(ap)
    ap.add_argument("--teachers_dir", default="/tmp/train_dir")
    ap.add_argument("--teachers_max_steps", type=int, default=3000)
    ap.add_argument("--nb_teachers", type=int, default=10)
    ap.add_argument("--stdnt_share", type=int, default=1000)
    ap.add_argument("--lap_scale", type=int, default=10)
    ap.add_argument("--save_labels", action="store_true")
    a = ap.parse_args(argv)
    return train_student(a, a.nb_teachers)


if __name__ == "__main__":
    main()
