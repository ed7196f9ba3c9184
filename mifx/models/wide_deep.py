"""Chicago-Taxi Wide&Deep model (DNNLinearCombinedClassifier equivalent).

Reference parity: ``airflow-dags/taxi_utils.py:148-191`` (`_build_estimator`) and
``trainer_fn`` (`taxi_utils.py:285-356`): DNN over the 3 z-scored dense floats with hidden units
``[max(2, int(100 * 0.7**i)) for i in range(4)] == [100, 70, 48, 34]``; linear part over
categorical identity columns (``default_value=0`` clamps out-of-range ids to bucket 0) — the
vocab features (1000 + 10 OOV buckets), the 4 bucketized lat/lon features (10 buckets) and the
``zip``-truncated categorical keys ``trip_start_hour/day/month`` with 24/31/12 buckets
(`taxi_utils.py:178-185`). Head: binary logistic (sigmoid cross-entropy).

Two implementations share one parameterisation:
  * :class:`WideDeepModel` — plain PyTorch (fp32), runs anywhere; the numerics reference.
  * the fused HIP step in :mod:`mifx.trainer.fused_wide_deep` (gfx950), which uses the padded
    "canonical" layout produced by :func:`pack_canonical` (biases folded into a constant-1 input
    column of every layer).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
from torch import nn

# ---- taxi feature contract (taxi_utils.py:32-67) ------------------------------------------
DENSE_FLOAT_FEATURE_KEYS = ["trip_miles", "fare", "trip_seconds"]
VOCAB_FEATURE_KEYS = ["payment_type", "company"]
BUCKET_FEATURE_KEYS = ["pickup_latitude", "pickup_longitude", "dropoff_latitude", "dropoff_longitude"]
CATEGORICAL_FEATURE_KEYS = [
    "trip_start_hour", "trip_start_day", "trip_start_month", "pickup_census_tract",
    "dropoff_census_tract", "pickup_community_area", "dropoff_community_area",
]
MAX_CATEGORICAL_FEATURE_VALUES = [24, 31, 12]
VOCAB_SIZE = 1000
OOV_SIZE = 10
FEATURE_BUCKET_COUNT = 10
LABEL_KEY = "tips"
FARE_KEY = "fare"


def transformed_name(key: str) -> str:
    return key + "_xf"


def wide_columns() -> list[tuple[str, int]]:
    """(transformed feature name, num_buckets) of the linear part, in kernel order."""
    cols = [(transformed_name(k), VOCAB_SIZE + OOV_SIZE) for k in VOCAB_FEATURE_KEYS]
    cols += [(transformed_name(k), FEATURE_BUCKET_COUNT) for k in BUCKET_FEATURE_KEYS]
    # zip() truncation of the 7 categorical keys to the 3 max values (taxi_utils.py:178-185)
    cols += [(transformed_name(k), nb) for k, nb in zip(CATEGORICAL_FEATURE_KEYS, MAX_CATEGORICAL_FEATURE_VALUES)]
    return cols


def dnn_hidden_units(first: int = 100, num_layers: int = 4, decay: float = 0.7) -> list[int]:
    return [max(2, int(first * decay ** i)) for i in range(num_layers)]


@dataclass
class WideDeepConfig:
    dense_features: list[str] = field(default_factory=lambda: [transformed_name(k) for k in DENSE_FLOAT_FEATURE_KEYS])
    wide: list[tuple[str, int]] = field(default_factory=wide_columns)
    hidden_units: list[int] = field(default_factory=dnn_hidden_units)
    label: str = transformed_name(LABEL_KEY)

    @property
    def wide_offsets(self) -> list[int]:
        out, o = [], 0
        for _, nb in self.wide:
            out.append(o)
            o += nb
        return out

    @property
    def wide_rows(self) -> int:
        return sum(nb for _, nb in self.wide)


# ---- record layout shared with csrc/wide_deep.hip --------------------------------------------
RECORD_DTYPE = np.dtype([("d", "<f4", (3,)), ("id", "<u2", (9,)), ("label", "<u2")])
assert RECORD_DTYPE.itemsize == 32


class WideDeepModel(nn.Module):
    """fp32 PyTorch Wide&Deep; TF initialisers (glorot-uniform kernels, zero biases/linear)."""

    def __init__(self, cfg: WideDeepConfig | None = None, seed: int | None = 0):
        super().__init__()
        self.cfg = cfg or WideDeepConfig()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        dims = [len(self.cfg.dense_features)] + list(self.cfg.hidden_units)
        self.dnn = nn.ModuleList(nn.Linear(dims[i], dims[i + 1]) for i in range(len(dims) - 1))
        self.head = nn.Linear(dims[-1], 1)
        for lin in list(self.dnn) + [self.head]:
            bound = math.sqrt(6.0 / (lin.in_features + lin.out_features))
            with torch.no_grad():
                lin.weight.copy_(torch.rand(lin.weight.shape, generator=g) * 2 * bound - bound)
                lin.bias.zero_()
        self.wide = nn.Parameter(torch.zeros(self.cfg.wide_rows))
        self.wide_bias = nn.Parameter(torch.zeros(1))
        self.register_buffer("wide_off", torch.tensor(self.cfg.wide_offsets, dtype=torch.long), persistent=False)
        self.register_buffer("wide_nb", torch.tensor([nb for _, nb in self.cfg.wide], dtype=torch.long),
                             persistent=False)

    def wide_index(self, ids: torch.Tensor) -> torch.Tensor:
        ids = ids.long()
        ids = torch.where((ids >= 0) & (ids < self.wide_nb), ids, torch.zeros_like(ids))
        return ids + self.wide_off

    def forward(self, dense: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
        h = dense.float()
        for lin in self.dnn:
            h = torch.relu(lin(h))
        deep = self.head(h).squeeze(-1)
        wide = self.wide[self.wide_index(ids)].sum(-1) + self.wide_bias
        return deep + wide

    def loss(self, dense, ids, labels, reduction: str = "sum") -> torch.Tensor:
        return nn.functional.binary_cross_entropy_with_logits(self(dense, ids), labels.float(), reduction=reduction)


# ---- canonical padded layout (must match csrc/wide_deep.hip) --------------------------------
LAYER_KN = [(32, 128), (128, 96), (96, 64), (64, 64), (64, 16)]
WTOT = sum(k * n for k, n in LAYER_KN)  # 27648
NWIDE = 2128
NTILE = 108
STRIDE = NTILE * 256 + 2176


def _offsets():
    off, tb, o, t = [], [], 0, 0
    for k, n in LAYER_KN:
        off.append(o)
        tb.append(t)
        o += k * n
        t += (n // 16) * (k // 16)
    return off, tb


LAYER_OFF, TILE_BASE = _offsets()


def _real_dims(cfg: WideDeepConfig) -> list[tuple[int, int]]:
    dims = [len(cfg.dense_features)] + list(cfg.hidden_units) + [1]
    return [(dims[i], dims[i + 1]) for i in range(len(dims) - 1)]


def check_fused_compatible(cfg: WideDeepConfig) -> None:
    real = _real_dims(cfg)
    if len(real) != len(LAYER_KN):
        raise ValueError("fused kernel is specialised for 4 hidden layers")
    for li, ((kr, nr), (k, n)) in enumerate(zip(real, LAYER_KN)):
        last = li == len(LAYER_KN) - 1
        if kr + 1 > k or (nr if last else nr + 1) > n:
            raise ValueError(f"layer {kr}->{nr} does not fit padded {k}x{n}")
    if [nb for _, nb in cfg.wide] != [1010, 1010, 10, 10, 10, 10, 24, 31, 12]:
        raise ValueError("fused kernel is specialised for the taxi wide columns")


WIDE_PAD = 2176


def _trainable_masks(cfg: WideDeepConfig) -> list[np.ndarray]:
    """Per layer [N, K] bool: real weights + folded biases (the trainable entries)."""
    out = []
    for (K, N), (kr, nr) in zip(LAYER_KN, _real_dims(cfg)):
        out.append((np.arange(N)[:, None] < nr) & (np.arange(K)[None, :] <= kr))
    return out


def compact_tile_map(cfg: WideDeepConfig | None = None, compact: bool = True) -> tuple[np.ndarray, int]:
    """(tmap int32 [NTILE], stride): tile -> position in the compact gradient slab, -1 for 16x16 dW tiles
    that hold only padding. The kernel skips those tiles when it writes its slab, so the slab write,
    the slab reduction and the DP all-reduce move ~1/3 fewer bytes (72 of 108 tiles are live for the
    taxi [100, 70, 48, 34] tower)."""
    cfg = cfg or WideDeepConfig()
    check_fused_compatible(cfg)
    if not compact:  # every tile stored (the full padded slab)
        return np.arange(NTILE, dtype=np.int32), STRIDE
    tmap = np.full(NTILE, -1, np.int32)
    c = 0
    for li, ((K, N), m) in enumerate(zip(LAYER_KN, _trainable_masks(cfg))):
        for nt in range(N // 16):
            for kt in range(K // 16):
                if m[16 * nt:16 * nt + 16, 16 * kt:16 * kt + 16].any():
                    tmap[TILE_BASE[li] + nt * (K // 16) + kt] = c
                    c += 1
    return tmap, c * 256 + WIDE_PAD


def stage_dims(cfg: WideDeepConfig | None = None) -> list[int]:
    """Live part of the padded bf16 weight image the fused kernel stages into LDS: per layer the rows
    that carry real weights or the constant-1 producer (n <= n_real; the head has no producer row) and
    the 16-byte granules up to the bias column k_real. -> rows[5] + granules_per_row[5]."""
    cfg = cfg or WideDeepConfig()
    check_fused_compatible(cfg)
    real = _real_dims(cfg)
    rows = [nr + (1 if li < len(real) - 1 else 0) for li, (_, nr) in enumerate(real)]
    gpr = [kr // 8 + 1 for kr, _ in real]
    return rows + gpr


def canonical_index_maps(cfg: WideDeepConfig | None = None, compact: bool = True):
    """Return (gidx int32 [WTOT+NWIDE], mask uint8 [WTOT+NWIDE]).

    gidx maps each canonical parameter to its position in the kernel's compact tile-native gradient
    slab (see compact_tile_map); mask marks trainable entries (real weights + folded biases). Entries
    of dead tiles are never trainable (gidx 0, mask 0)."""
    cfg = cfg or WideDeepConfig()
    tmap, stride = compact_tile_map(cfg, compact)
    gidx = np.zeros(WTOT + NWIDE, np.int32)
    mask = np.zeros(WTOT + NWIDE, np.uint8)
    for li, ((K, N), m) in enumerate(zip(LAYER_KN, _trainable_masks(cfg))):
        n = np.arange(N)[:, None]
        k = np.arange(K)[None, :]
        ct = tmap[TILE_BASE[li] + (n // 16) * (K // 16) + (k // 16)]
        lane = 16 * ((n % 16) // 4) + (k % 16)
        idx = np.where(ct >= 0, ct * 256 + (n % 4) * 64 + lane, 0)
        assert (ct[m] >= 0).all()
        gidx[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = idx.reshape(-1)
        mask[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = m.reshape(-1)
    gidx[WTOT:] = stride - WIDE_PAD + np.arange(NWIDE)
    mask[WTOT:] = 1
    return gidx, mask


def pack_canonical(model: WideDeepModel) -> np.ndarray:
    """torch model -> fp32 canonical parameter vector [WTOT + NWIDE]."""
    check_fused_compatible(model.cfg)
    out = np.zeros(WTOT + NWIDE, np.float32)
    lins = list(model.dnn) + [model.head]
    for li, ((K, N), lin) in enumerate(zip(LAYER_KN, lins)):
        wt = np.zeros((N, K), np.float32)
        nr, kr = lin.weight.shape
        wt[:nr, :kr] = lin.weight.detach().cpu().numpy()
        wt[:nr, kr] = lin.bias.detach().cpu().numpy()
        if li < len(LAYER_KN) - 1:
            wt[nr, kr] = 1.0  # produces the constant-1 column of the next layer's input
        out[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = wt.reshape(-1)
    nw = model.wide.numel()
    out[WTOT:WTOT + nw] = model.wide.detach().cpu().numpy()
    out[WTOT + nw] = float(model.wide_bias.detach().cpu().item())
    return out


def unpack_canonical(vec, model: WideDeepModel) -> WideDeepModel:
    """fp32 canonical vector -> torch model parameters (in place)."""
    vec = np.asarray(vec.detach().cpu() if torch.is_tensor(vec) else vec, dtype=np.float32)
    lins = list(model.dnn) + [model.head]
    with torch.no_grad():
        for li, ((K, N), lin) in enumerate(zip(LAYER_KN, lins)):
            wt = vec[LAYER_OFF[li]:LAYER_OFF[li] + K * N].reshape(N, K)
            nr, kr = lin.weight.shape
            lin.weight.copy_(torch.from_numpy(wt[:nr, :kr].copy()))
            lin.bias.copy_(torch.from_numpy(wt[:nr, kr].copy()))
        nw = model.wide.numel()
        model.wide.copy_(torch.from_numpy(vec[WTOT:WTOT + nw].copy()))
        model.wide_bias.fill_(float(vec[WTOT + nw]))
    return model


def canonical_grad_to_torch(grad_tile_native: np.ndarray, model: WideDeepModel,
                            gidx: np.ndarray | None = None) -> dict[str, np.ndarray]:
    """Map a tile-native gradient slab back to named torch-shaped gradients (for tests). gidx: the kernel's
    canonical -> slab map (default: the tile kernel's compact layout)."""
    if gidx is None:
        gidx, _ = canonical_index_maps(model.cfg)
    canon = np.asarray(grad_tile_native)[gidx]
    out = {}
    lins = list(model.dnn) + [model.head]
    names = [f"dnn.{i}" for i in range(len(model.dnn))] + ["head"]
    for li, ((K, N), lin, nm) in enumerate(zip(LAYER_KN, lins, names)):
        wt = canon[LAYER_OFF[li]:LAYER_OFF[li] + K * N].reshape(N, K)
        nr, kr = lin.weight.shape
        out[nm + ".weight"] = wt[:nr, :kr]
        out[nm + ".bias"] = wt[:nr, kr]
    nw = model.wide.numel()
    out["wide"] = canon[WTOT:WTOT + nw]
    out["wide_bias"] = canon[WTOT + nw:WTOT + nw + 1]
    return out


def records_to_tensors(rec: np.ndarray | torch.Tensor):
    """Decode packed 32-B records into (dense f32 [N,3], ids int64 [N,9], label f32 [N])."""
    if torch.is_tensor(rec):
        raw = rec.view(torch.uint8).reshape(-1, 32)
        dense = raw[:, :12].contiguous().view(torch.float32).reshape(-1, 3)
        u16 = raw[:, 12:32].contiguous().view(torch.int16).reshape(-1, 10).to(torch.int32) & 0xFFFF
        return dense, u16[:, :9].long(), u16[:, 9].float()
    rec = np.asarray(rec).view(RECORD_DTYPE)
    return (torch.from_numpy(rec["d"].copy()), torch.from_numpy(rec["id"].astype(np.int64)),
            torch.from_numpy(rec["label"].astype(np.float32)))


def pack_transformed_columns(cols: dict, cfg: WideDeepConfig | None = None, with_label: bool = True) -> np.ndarray:
    """Transform outputs (dict of columns, `taxi_utils.py:106-145` names) -> packed 32-B records."""
    cfg = cfg or WideDeepConfig()
    n = len(next(iter(cols.values())))
    dense = np.stack([np.asarray(cols[k], np.float32) for k in cfg.dense_features], 1) if n else np.zeros((0, 3))
    ids = np.stack([np.asarray(cols[k], np.int64) for k, _ in cfg.wide], 1) if n else np.zeros((0, 9))
    label = np.asarray(cols[cfg.label], np.int64) if with_label and cfg.label in cols else np.zeros(n, np.int64)
    return tensors_to_records(dense, ids, label)


def tensors_to_records(dense, ids, label) -> np.ndarray:
    n = len(label)
    rec = np.zeros(n, RECORD_DTYPE)
    rec["d"] = np.asarray(dense, np.float32).reshape(n, 3)
    rec["id"] = np.clip(np.asarray(ids), 0, 65535).astype(np.uint16)
    rec["label"] = np.asarray(label).astype(np.uint16)
    return rec


# ---- register-chained kernel layout (csrc/wd_chain.hip) ---------------------------------------
# The chained kernel feeds layer l's MFMA output tiles straight into layer l+1 as its B operand, so layer
# l+1's k axis is consumed in "C order": inside every 32-block, position 8H + E holds feature
# 16 (E // 4) + 4 H + E % 4. Its LDS weight image W_l^T [N][K] therefore has natural rows and C-ordered
# columns. Image row n sits at physical row wperm(n) (bit 4 of n flips bit 2) and rows are padded by CHAIN_PAD
# elements (the kernel's WPAD) -- together conflict-free LDS reads (see the kernel's wperm note). dW tiles come
# out with C-order k columns and, for layers 1-4, an n axis in "C o C" order: the kernel stages the dZ fragments
# it holds (C positions of the layer above's k axis) as 16-byte pairs, which applies chain_perm once more.
CHAIN_PAD = 16
CHAIN_LW = [int(v) for v in np.cumsum([0] + [n * (k + CHAIN_PAD) for k, n in LAYER_KN])[:-1]]
CHAIN_LWEND = sum(n * (k + CHAIN_PAD) for k, n in LAYER_KN)  # 33536


def chain_perm(K: int) -> np.ndarray:
    """f[c] = natural feature held at C-order position c of a K-wide (K % 32 == 0) chained input axis."""
    c = np.arange(K)
    return 32 * (c // 32) + 16 * ((c % 8) // 4) + 4 * ((c % 32) // 8) + c % 4


def chain_wperm(n: np.ndarray) -> np.ndarray:
    """Physical LDS row of weight-image row n (the kernel's wperm)."""
    return n ^ (((n >> 4) & 1) << 2)


def chain_dw_rows(li: int) -> np.ndarray:
    """f[j] = natural output feature on row j of layer li's dW tiles."""
    N = LAYER_KN[li][1]
    if li == len(LAYER_KN) - 1:
        return np.arange(N)  # dZ5 is staged in natural order
    c = chain_perm(N)
    return c[c]


def chain_image_offsets(li: int) -> np.ndarray:
    """[N, K] element offsets in the chained kernel's weight image of layer li's entry (row n, C position c)."""
    K, N = LAYER_KN[li]
    n = np.arange(N)[:, None]
    c = np.arange(K)[None, :]
    return CHAIN_LW[li] + chain_wperm(n) * (K + CHAIN_PAD) + c


def chain_image(param) -> np.ndarray:
    """fp32 canonical vector -> fp32 weight image in the chained kernel's LDS layout [CHAIN_LWEND]
    (cast to bf16 on the device)."""
    p = np.asarray(param.detach().cpu() if torch.is_tensor(param) else param, dtype=np.float32)
    img = np.zeros(CHAIN_LWEND, np.float32)
    for li, (K, N) in enumerate(LAYER_KN):
        w = p[LAYER_OFF[li]:LAYER_OFF[li] + K * N].reshape(N, K)
        img[chain_image_offsets(li)] = w[:, chain_perm(K)]
    return img


def chain_maps(cfg: WideDeepConfig | None = None):
    """Index maps of the chained kernel: (tmap int32 [NTILE], stride, gidx int32 [WTOT+NWIDE],
    mask uint8 [WTOT+NWIDE], wmap int32 [WTOT]).

    tmap: dW tile (rows chain_dw_rows, C-order columns; id TILE_BASE + nt * K/16 + kt) -> compact slab position (-1: only
    padding); gidx: canonical parameter -> slab position (tile-native order inside a tile, as wd_fused);
    wmap: canonical DNN parameter -> offset in the bf16 image the optimizer re-emits."""
    cfg = cfg or WideDeepConfig()
    check_fused_compatible(cfg)
    masks = _trainable_masks(cfg)
    tmap = np.full(NTILE, -1, np.int32)
    c = 0
    for li, ((K, N), m) in enumerate(zip(LAYER_KN, masks)):
        mi = m[chain_dw_rows(li)][:, chain_perm(K)]  # dW tile coordinates
        for nt in range(N // 16):
            for kt in range(K // 16):
                if mi[16 * nt:16 * nt + 16, 16 * kt:16 * kt + 16].any():
                    tmap[TILE_BASE[li] + nt * (K // 16) + kt] = c
                    c += 1
    stride = c * 256 + WIDE_PAD
    gidx = np.zeros(WTOT + NWIDE, np.int32)
    mask = np.zeros(WTOT + NWIDE, np.uint8)
    wmap = np.zeros(WTOT, np.int32)
    for li, ((K, N), m) in enumerate(zip(LAYER_KN, masks)):
        cinv = np.argsort(chain_perm(K))  # natural k -> image column
        n = np.arange(N)[:, None]
        col = cinv[None, :].repeat(N, 0)
        j = np.argsort(chain_dw_rows(li))[n]  # natural n -> dW tile row
        ct = tmap[TILE_BASE[li] + (j // 16) * (K // 16) + col // 16]
        lane = 16 * ((j % 16) // 4) + col % 16
        idx = np.where(ct >= 0, ct * 256 + (j % 4) * 64 + lane, 0)
        assert (ct[m] >= 0).all()
        gidx[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = idx.reshape(-1)
        mask[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = m.reshape(-1)
        wmap[LAYER_OFF[li]:LAYER_OFF[li] + K * N] = chain_image_offsets(li)[n, col].reshape(-1)
    gidx[WTOT:] = stride - WIDE_PAD + np.arange(NWIDE)
    mask[WTOT:] = 1
    return tmap, stride, gidx, mask, wmap
