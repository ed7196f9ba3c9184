"""KFP taxi DNN classifier: indicator (one-hot) columns + numeric columns -> hidden layer(s) -> 1 logit.

Reference: `kubeflow-pipelines/taxi/preprocessing.py:26-124` (feature columns) and the dnntrainer
component args (`taxi-cab-classification-pipeline.py:55-57,117-126`: hidden_layer_size '1500',
Adagrad lr 0.1, 3,000 steps). The 6,170-wide input is:
  6 vocab features x (1000 + 10 OOV) + hour 24 + day 31 + month 12 + 4 lat/lon buckets x 10 + 3 numeric.
`W1` is stored row-major [6170, H] so an indicator input is a row gather (see csrc/embag_mlp.hip)."""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn as nn

VOCAB_FEATURE_KEYS = ["pickup_census_tract", "dropoff_census_tract", "payment_type", "company",
                      "pickup_community_area", "dropoff_community_area"]
CATEGORICAL_FEATURE_KEYS = ["trip_start_hour", "trip_start_day", "trip_start_month"]
MAX_CATEGORICAL_FEATURE_VALUES = [24, 31, 12]
BUCKET_FEATURE_KEYS = ["pickup_latitude", "pickup_longitude", "dropoff_latitude", "dropoff_longitude"]
DENSE_FLOAT_FEATURE_KEYS = ["trip_miles", "fare", "trip_seconds"]
VOCAB_SIZE, OOV_SIZE, FEATURE_BUCKET_COUNT = 1000, 10, 10
LABEL_KEY = "tips"


@dataclass
class TaxiDNNConfig:
    sparse: list = field(default_factory=lambda: [(k, VOCAB_SIZE + OOV_SIZE) for k in VOCAB_FEATURE_KEYS]
                         + list(zip(CATEGORICAL_FEATURE_KEYS, MAX_CATEGORICAL_FEATURE_VALUES))
                         + [(k, FEATURE_BUCKET_COUNT) for k in BUCKET_FEATURE_KEYS])
    dense: list = field(default_factory=lambda: list(DENSE_FLOAT_FEATURE_KEYS))
    hidden: int = 1500
    label: str = LABEL_KEY

    @property
    def offsets(self) -> np.ndarray:
        sizes = [n for _, n in self.sparse]
        return np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)

    @property
    def sparse_rows(self) -> int:
        return int(sum(n for _, n in self.sparse))

    @property
    def input_dim(self) -> int:
        return self.sparse_rows + len(self.dense)


class TaxiDNN(nn.Module):
    def __init__(self, cfg: TaxiDNNConfig | None = None, seed: int | None = 0, hidden: int | None = None):
        super().__init__()
        self.cfg = cfg or TaxiDNNConfig()
        if hidden is not None:
            self.cfg.hidden = int(hidden)
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        fan_in, H = self.cfg.input_dim, self.cfg.hidden
        lim1 = (6.0 / (fan_in + H)) ** 0.5  # glorot uniform (tf.layers.dense default)
        self.W1 = nn.Parameter((torch.rand(fan_in, H, generator=g) * 2 - 1) * lim1)
        self.b1 = nn.Parameter(torch.zeros(H))
        lim2 = (6.0 / (H + 1)) ** 0.5
        self.w2 = nn.Parameter((torch.rand(H, generator=g) * 2 - 1) * lim2)
        self.b2 = nn.Parameter(torch.zeros(1))
        self.register_buffer("offsets", torch.as_tensor(self.cfg.offsets))

    def rows(self, ids: torch.Tensor) -> torch.Tensor:
        """ids [B, F] per-feature indices -> global W1 rows [B, F] (clamped into each feature's range)."""
        sizes = torch.as_tensor([n for _, n in self.cfg.sparse], device=ids.device)
        return ids.clamp(min=0).minimum(sizes - 1) + self.offsets.to(ids.device)

    def forward(self, ids: torch.Tensor, dense: torch.Tensor) -> torch.Tensor:
        z = self.b1 + self.W1[self.rows(ids)].sum(1) + dense @ self.W1[self.cfg.sparse_rows:]
        return torch.relu(z) @ self.w2 + self.b2

    def loss(self, ids, dense, label, reduction: str = "sum"):
        return nn.functional.binary_cross_entropy_with_logits(self(ids, dense), label.float(), reduction=reduction)


def columns_to_tensors(cols: dict, cfg: TaxiDNNConfig, with_label: bool = True):
    """Transformed column dict -> (ids int64 [N, F], dense float32 [N, D], label float32 [N] | None)."""
    ids = np.stack([np.nan_to_num(np.asarray(cols[k], dtype=np.float64), nan=0).astype(np.int64)
                    for k, _ in cfg.sparse], 1)
    dense = np.stack([np.nan_to_num(np.asarray(cols[k], dtype=np.float64), nan=0.0) for k in cfg.dense], 1)
    y = None
    if with_label and cfg.label in cols:
        y = torch.from_numpy(np.asarray(cols[cfg.label]).astype(np.float32))
    return torch.from_numpy(ids), torch.from_numpy(dense.astype(np.float32)), y
