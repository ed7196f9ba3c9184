"""PATE teacher-vote aggregation (reference: `research/pate_2017/aggregation.py:22-130`).

`noisy_max` runs on the GPU as one kernel (register bincount + Philox Laplace/Gaussian noise +
argmax per sample, csrc/dp.hip) instead of the reference's per-sample Python loop; on CPU the
bit-identical host implementation in `mifx.ops.dp` runs."""
from __future__ import annotations

import numpy as np

from ...ops import dp as dpops


def labels_from_probs(probs) -> np.ndarray:
    """Argmax over the last axis -> int32 labels."""
    return np.asarray(np.argmax(np.asarray(probs), axis=-1), dtype=np.int32)


def noisy_max(logits, lap_scale: float, return_clean_votes: bool = False, num_classes: int = 10, seed: int = 0,
              offset: int = 0, device=None):
    """Teacher outputs [T, N, C] (probs/logits) or labels [T, N] -> noisy-argmax labels [N] (int32).

    With `return_clean_votes`: (labels, clean_votes [N, C], teacher_labels [T, N])."""
    arr = np.asarray(logits)
    labels = labels_from_probs(arr) if arr.ndim == 3 else arr.astype(np.int32)
    if arr.ndim == 3:
        num_classes = arr.shape[-1]
    res = dpops.noisy_max(labels, num_classes, lap_scale, "laplace", seed, offset, return_clean_votes, device)
    if return_clean_votes:
        out, votes = res
        return out, votes, labels
    return res


def gnmax(labels, num_classes: int, sigma: float, seed: int = 0, offset: int = 0, device=None) -> np.ndarray:
    """Gaussian NoisyMax (PATE-2018): argmax(votes + N(0, sigma^2))."""
    return dpops.noisy_max(np.asarray(labels, np.int32), num_classes, sigma, "gaussian", seed, offset, False, device)


def confident_gnmax(labels, num_classes: int, threshold: float, sigma1: float, sigma2: float, seed: int = 0,
                    offset: int = 0, device=None):
    """Confident-GNMax (PATE-2018 Alg. 1): answer only where max vote + N(0, sigma1^2) >= threshold.
    Returns (answered mask [N], labels [N] (-1 where unanswered))."""
    lab = np.asarray(labels, np.int32)
    T, N = lab.shape
    votes = np.zeros((N, num_classes), np.int32)
    for t in range(T):
        np.add.at(votes, (np.arange(N), lab[t]), 1)
    rng_noise = dpops.noise_reference_pate(N, 1, sigma1, 1, seed ^ 0x5BD1E995, offset)[:, 0]
    answered = votes.max(axis=1) + rng_noise >= threshold
    out = np.full(N, -1, np.int32)
    if answered.any():
        out[answered] = gnmax(lab[:, answered], num_classes, sigma2, seed, offset, device)
    return answered, out


def aggregation_most_frequent(logits) -> np.ndarray:
    """Noise-free plurality vote."""
    arr = np.asarray(logits)
    labels = labels_from_probs(arr) if arr.ndim == 3 else arr.astype(np.int32)
    C = arr.shape[-1] if arr.ndim == 3 else int(labels.max()) + 1
    votes = np.zeros((labels.shape[1], max(C, 10)), np.int32)
    for t in range(labels.shape[0]):
        np.add.at(votes, (np.arange(labels.shape[1]), labels[t]), 1)
    return np.argmax(votes, axis=1).astype(np.int32)


def accuracy(logits_or_labels, labels) -> float:
    """Fraction correct (reference `pate_2017/metrics.py:22-49`)."""
    a = np.asarray(logits_or_labels)
    pred = np.argmax(a, axis=1) if a.ndim == 2 else a
    return float(np.mean(pred.astype(np.int64) == np.asarray(labels).astype(np.int64)))
