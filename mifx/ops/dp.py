"""DP-SGD aggregation and PATE noisy-max kernels (csrc/dp.hip) with exact host references.

The noise streams are Philox4x32-10 keyed by `seed` and offset by `offset` (both 64-bit); the
numpy implementation below reproduces the device bits, so CPU and GPU results agree to float
rounding of log/sincos. On a CUDA/HIP device the native kernels are required."""
from __future__ import annotations

import functools

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, VP, check, ptr, sig, stream_handle

U64 = __import__("ctypes").c_ulonglong


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("dp")
    return {
        "clip": sig(lib, "mifx_dp_clip_sum_noise", [VP, I32, I32, I32, F32, F32, F32, U64, U64, VP, VP, VP, VP]),
        "chunk": sig(lib, "mifx_dp_chunk", []),
        "maxrows": sig(lib, "mifx_dp_max_rows", []),
        "noisy_max": sig(lib, "mifx_pate_noisy_max", [VP, I32, I32, I32, F32, I32, U64, U64, VP, VP, VP]),
        "maxc": sig(lib, "mifx_pate_max_classes", []),
    }


# ---- Philox4x32-10 (bit-exact with the device) --------------------------------------------------
_M0, _M1, _W0, _W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox4x32(c0, c1, c2, c3, seed: int) -> tuple:
    """Vectorised Philox4x32-10: counters are uint32 arrays (broadcastable); returns 4 uint32 arrays."""
    c = [np.asarray(x, np.uint32) for x in np.broadcast_arrays(c0, c1, c2, c3)]
    k0, k1 = np.uint32(seed & 0xFFFFFFFF), np.uint32((seed >> 32) & 0xFFFFFFFF)
    mask = np.uint64(0xFFFFFFFF)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c[0].astype(np.uint64)
            p1 = _M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & mask).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & mask).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return tuple(c)


def _u01(v):
    return ((v >> np.uint32(8)).astype(np.float32) + np.float32(1.0)) * np.float32(1.0 / 16777216.0)


def _box_muller(a, b):
    r = np.sqrt(np.float32(-2.0) * np.log(_u01(a)))
    t = np.float32(6.283185307179586) * _u01(b)
    return (r * np.cos(t)).astype(np.float32), (r * np.sin(t)).astype(np.float32)


def gaussian_noise_reference(n: int, seed: int, offset: int) -> np.ndarray:
    """The N(0,1) stream dp_clip_sum_noise adds to columns [0, n)."""
    q = np.arange((n + 3) // 4, dtype=np.uint32)
    x, y, z, w = philox4x32(q, 0, offset & 0xFFFFFFFF, (offset >> 32) & 0xFFFFFFFF, seed)
    z0, z1 = _box_muller(x, y)
    z2, z3 = _box_muller(z, w)
    return np.stack([z0, z1, z2, z3], axis=1).reshape(-1)[:n]


def _pad4(G: torch.Tensor) -> torch.Tensor:
    P = G.shape[1]
    return G if P % 4 == 0 else F.pad(G, (0, 4 - P % 4))


def clip_sum_noise(G: torch.Tensor, l2_norm_clip: float, stddev: float, denominator: float = 1.0, seed: int = 0,
                   offset: int = 0, return_norms: bool = False, out: torch.Tensor | None = None):
    """sum_m min(1, C/||G_m||) G_m + stddev * N(0, I), divided by `denominator` (GPU: written into `out` when
    given).

    G: [M, P] float32 per-microbatch (flattened, concatenated) gradients."""
    if G.dim() != 2:
        raise ValueError("G must be [num_microbatches, num_params]")
    M, P = G.shape
    if G.device.type != "cuda":
        Gd = G.double()
        norms = Gd.norm(dim=1)
        scale = torch.where(norms > l2_norm_clip, l2_norm_clip / norms.clamp_min(1e-300), torch.ones_like(norms))
        s = (Gd * scale[:, None]).sum(0)
        if stddev:
            s = s + stddev * torch.from_numpy(gaussian_noise_reference(P, seed, offset)).double()
        out = (s / denominator).float()
        return (out, norms.float()) if return_norms else out
    fns = _fns()
    if M > fns["maxrows"]():
        raise ValueError(f"at most {fns['maxrows']()} microbatches per call")
    Gp = _pad4(G.float().contiguous())
    ld = Gp.shape[1]
    nchunk = (ld + fns["chunk"]() - 1) // fns["chunk"]()
    partial = torch.empty(M * nchunk, dtype=torch.float32, device=G.device)
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=G.device)
    elif out.dtype != torch.float32 or out.numel() != P or not out.is_contiguous() or out.device != G.device:
        raise ValueError("out must be a contiguous float32 tensor of G.shape[1] elements on G's device")
    norms = torch.empty(M, dtype=torch.float32, device=G.device) if return_norms else None
    check(fns["clip"](ptr(Gp), M, ld, P, float(l2_norm_clip), float(stddev), float(denominator), seed, offset,
                      ptr(partial), ptr(out), ptr(norms), stream_handle(G.device)), "mifx_dp_clip_sum_noise")
    return (out, norms) if return_norms else out


def noise_reference_pate(N: int, C: int, scale: float, mode: int, seed: int, offset: int) -> np.ndarray:
    """[N, C] noise the device adds to vote counts (mode 0 Laplace(scale), mode 1 N(0, scale^2))."""
    i = np.arange(N, dtype=np.uint32)[:, None]
    c0 = np.arange(0, C, 4, dtype=np.uint32)[None, :]
    r = philox4x32(i, c0, offset & 0xFFFFFFFF, (offset >> 32) & 0xFFFFFFFF, seed)
    if mode == 0:
        cols = []
        for v in r:
            u = _u01(v) - np.float32(0.5)
            cols.append(-np.float32(scale) * np.sign(u) * np.log(np.maximum(np.float32(1) - 2 * np.abs(u),
                                                                             np.float32(1e-30))))
        n = np.stack(cols, axis=2)
    else:
        z0, z1 = _box_muller(r[0], r[1])
        z2, z3 = _box_muller(r[2], r[3])
        n = np.stack([z0, z1, z2, z3], axis=2) * np.float32(scale)
    return n.reshape(N, -1)[:, :C].astype(np.float32)


def noisy_max(labels, num_classes: int, noise_scale: float, mode: str = "laplace", seed: int = 0, offset: int = 0,
              return_clean_votes: bool = False, device=None):
    """PATE aggregation: per-sample teacher vote counts + noise, argmax. labels: [T, N] int."""
    m = {"laplace": 0, "gaussian": 1}[mode]
    lab = torch.as_tensor(np.asarray(labels) if not torch.is_tensor(labels) else labels).to(torch.int32)
    T, N = lab.shape
    dev = torch.device(device) if device is not None else lab.device
    if dev.type != "cuda":
        ln = lab.cpu().numpy()
        votes = np.zeros((N, num_classes), np.int32)
        for t in range(T):
            np.add.at(votes, (np.arange(N), ln[t]), 1)
        noisy = votes.astype(np.float32) + noise_reference_pate(N, num_classes, noise_scale, m, seed, offset)
        res = np.argmax(noisy, axis=1).astype(np.int32)
        return (res, votes) if return_clean_votes else res
    fns = _fns()
    if num_classes > fns["maxc"]():
        raise ValueError(f"at most {fns['maxc']()} classes")
    lab = lab.to(dev).contiguous()
    out = torch.empty(N, dtype=torch.int32, device=dev)
    clean = torch.empty(N, num_classes, dtype=torch.int32, device=dev) if return_clean_votes else None
    check(fns["noisy_max"](ptr(lab), T, N, num_classes, float(noise_scale), m, seed, offset, ptr(out), ptr(clean),
                           stream_handle(dev)), "mifx_pate_noisy_max")
    res = out.cpu().numpy()
    return (res, clean.cpu().numpy()) if return_clean_votes else res
