"""Synthetic Chicago-Taxi-shaped data (post-Transform feature space and raw CSV space).

There is no network for the real dataset, so benchmarks use records with the exact shape of
the Transform output consumed by the trainer (`taxi_utils.py:106-145`): 3 z-scored floats,
2 vocab ids in [0, 1010), 4 bucket ids in [0, 10), hour/day/month, binary label. Labels come
from a fixed random "teacher" so training has a learnable signal.
"""
from __future__ import annotations

import numpy as np
import torch

from ..models.wide_deep import RECORD_DTYPE


def _teacher(gen: torch.Generator):
    w_dense = torch.randn(3, generator=gen) * 0.8
    w_vocab = torch.randn(2, 1010, generator=gen) * 0.5
    w_bucket = torch.randn(4, 10, generator=gen) * 0.3
    w_hour = torch.randn(24, generator=gen) * 0.4
    return w_dense, w_vocab, w_bucket, w_hour


def synthetic_records(n: int, device="cpu", seed: int = 0, chunk: int = 1 << 22) -> torch.Tensor:
    """Packed 32-B records [n, 32] uint8 on `device` (generated in chunks on that device)."""
    device = torch.device(device)
    gen_cpu = torch.Generator().manual_seed(seed)
    teacher = [t.to(device) for t in _teacher(gen_cpu)]
    out = torch.empty((n, 32), dtype=torch.uint8, device=device)
    g = torch.Generator(device=device).manual_seed(seed + 1)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        dense = torch.randn(m, 3, generator=g, device=device)
        # zipf-like vocab popularity: sample u^3 so low ids dominate (like frequency-ranked vocab)
        u = torch.rand(m, 2, generator=g, device=device)
        vocab = (u.pow(3) * 1010).long().clamp_max(1009)
        buckets = torch.randint(0, 10, (m, 4), generator=g, device=device)
        hour = torch.randint(0, 24, (m, 1), generator=g, device=device)
        day = torch.randint(1, 32, (m, 1), generator=g, device=device)  # 31 -> clamps to bucket 0
        month = torch.randint(1, 13, (m, 1), generator=g, device=device)
        wd, wv, wb, wh = teacher
        logit = dense @ wd + wv[0][vocab[:, 0]] + wv[1][vocab[:, 1]] - 0.3
        logit = logit + wb.gather(1, buckets.t()).sum(0) + wh[hour[:, 0]]
        label = (torch.rand(m, generator=g, device=device) < torch.sigmoid(logit)).to(torch.int32)
        ids = torch.cat([vocab, buckets, hour, day, month], 1).to(torch.int32)
        u16 = torch.cat([ids, label[:, None]], 1).to(torch.int16)  # values < 32768
        rec = out[s:s + m]
        rec[:, :12] = dense.contiguous().view(torch.uint8).reshape(m, 12)
        rec[:, 12:32] = u16.contiguous().view(torch.uint8).reshape(m, 20)
    return out


def synthetic_records_np(n: int, seed: int = 0) -> np.ndarray:
    return synthetic_records(n, "cpu", seed).numpy().view(RECORD_DTYPE).reshape(-1)


TAXI_COLUMNS = [
    "pickup_community_area", "fare", "trip_start_month", "trip_start_hour", "trip_start_day",
    "trip_start_timestamp", "pickup_latitude", "pickup_longitude", "dropoff_latitude", "dropoff_longitude",
    "trip_miles", "pickup_census_tract", "dropoff_census_tract", "payment_type", "company", "trip_seconds",
    "dropoff_community_area", "tips",
]

_COMPANIES = [f"Company {i:03d}" for i in range(150)]
_PAYMENTS = ["Cash", "Credit Card", "No Charge", "Dispute", "Unknown", "Prcard"]


def synthetic_taxi_csv_rows(n: int, seed: int = 0, missing_rate: float = 0.02) -> list[dict]:
    """Raw CSV-shaped rows (18 columns of `airflow-dags/data/taxi_data/data.csv:1`), with missing
    values, for pipeline tests."""
    rng = np.random.default_rng(seed)
    rows = []
    for _ in range(n):
        miles = float(rng.gamma(2.0, 1.5))
        secs = int(max(60, miles * 200 + rng.normal(0, 120)))
        fare = round(3.25 + miles * 2.25 + rng.normal(0, 1.0), 2)
        pay = _PAYMENTS[min(len(_PAYMENTS) - 1, int(rng.exponential(0.8)))]
        tip = round(max(0.0, fare * (0.22 if pay == "Credit Card" else 0.01) + rng.normal(0, 0.8)), 2)
        r = {
            "pickup_community_area": int(rng.integers(1, 78)),
            "fare": fare,
            "trip_start_month": int(rng.integers(1, 13)),
            "trip_start_hour": int(rng.integers(0, 24)),
            "trip_start_day": int(rng.integers(1, 8)),
            "trip_start_timestamp": int(1.38e9 + rng.integers(0, 1e8)),
            "pickup_latitude": round(41.88 + rng.normal(0, 0.05), 6),
            "pickup_longitude": round(-87.63 + rng.normal(0, 0.05), 6),
            "dropoff_latitude": round(41.88 + rng.normal(0, 0.05), 6),
            "dropoff_longitude": round(-87.63 + rng.normal(0, 0.05), 6),
            "trip_miles": round(miles, 2),
            "pickup_census_tract": int(17031000000 + rng.integers(0, 9999)),
            "dropoff_census_tract": int(17031000000 + rng.integers(0, 9999)),
            "payment_type": pay,
            "company": _COMPANIES[min(len(_COMPANIES) - 1, int(rng.exponential(20)))],
            "trip_seconds": secs,
            "dropoff_community_area": int(rng.integers(1, 78)),
            "tips": tip,
        }
        for k in list(r):
            if k not in ("tips", "trip_start_hour", "trip_start_day", "trip_start_month") and rng.random() < missing_rate:
                r[k] = None
        rows.append(r)
    return rows


def synthetic_images(n: int, shape=(28, 28), num_classes: int = 10, seed: int = 0, channels: int = 1,
                     noise: float = 0.35):
    """MNIST/SVHN/CIFAR-shaped images with a learnable class signal (no dataset downloads offline):
    each class owns a fixed random smooth template; samples are template + noise, clipped to [0, 1].
    Returns (float32 [n, C, H, W] or [n, H, W] when channels == 1, int64 labels [n])."""
    g = torch.Generator().manual_seed(seed)
    h, w = shape
    base = torch.rand(num_classes, channels, h // 4 + 1, w // 4 + 1, generator=g)
    templates = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    x = templates[labels] + noise * torch.randn(n, channels, h, w, generator=g)
    x = x.clamp_(0.0, 1.0)
    return (x[:, 0] if channels == 1 else x), labels
