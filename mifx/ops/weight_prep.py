"""Per-step bf16 weight images of the GEMM-shaped convolutions, refreshed in ONE launch (csrc/weight_prep.hip).

`WeightPrep(params)` allocates, for each registered fp32 convolution weight, the bf16 images the implicit-GEMM kernels
read -- 1x1: [Cout, C] and its transpose [C, Cout] (input gradient); 3x3: [Cout, 9 C] (the channels_last storage)
and the flipped transpose [C, 9 Cout] -- and a device job table. `refresh()` (once per step, after the optimizer and
before the forward; inside a captured step it is one graph node) rewrites all of them. mifx.ops.conv1x1 / conv3x3 use
an image only while the weight's version counter still equals the one recorded at the refresh, so a weight updated
without a refresh falls back to a per-call cast."""
from __future__ import annotations

import ctypes
import functools

import torch

from . import _lib
from ._lib import I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("weight_prep")
    return {"job_bytes": sig(lib, "mifx_weight_prep_job_bytes", []),
            "job": sig(lib, "mifx_weight_prep_job", [VP, I32, VP, VP, I64, I32, I32, I32, I32, I32]),
            "run": sig(lib, "mifx_weight_prep", [VP, I32, I32, VP])}


_ACTIVE: dict = {}  # id(weight) -> (weight, version, images)


def images(w: torch.Tensor):
    """The refreshed bf16 images of w -- (fwd, bwd) -- or None (not registered / stale)."""
    e = _ACTIVE.get(id(w))
    if e is None or e[0] is not w or e[1] != w._version:
        return None
    return e[2]


class WeightPrep:
    def __init__(self, weights):
        self.weights = [w for w in weights if self.supported(w)]
        if not self.weights:
            raise ValueError("no supported convolution weights")
        dev = self.weights[0].device
        f = _fns()
        jb = f["job_bytes"]()
        recs, items, self.images = [], 0, []

        def job(kind, src, dst, n=0, R=0, C=0, sld=0, dld=0):
            nonlocal items
            buf = (ctypes.c_ubyte * jb)()
            k = f["job"](buf, kind, src, dst, n, R, C, sld, dld, items)
            if k <= 0:
                raise ValueError("weight_prep: bad job")
            recs.append(bytes(buf))
            items += k

        for w in self.weights:
            cout, c, kh, kw = w.shape
            if kh == 1:
                fwd = torch.empty(cout, c, device=dev, dtype=torch.bfloat16)
                bwd = torch.empty(c, cout, device=dev, dtype=torch.bfloat16)
                job(0, w.data_ptr(), fwd.data_ptr(), n=w.numel())
                job(1, w.data_ptr(), bwd.data_ptr(), R=cout, C=c, sld=c, dld=cout)
            else:  # 3x3, channels_last storage [Cout][3][3][C]
                fwd = torch.empty(cout, 9 * c, device=dev, dtype=torch.bfloat16)
                bwd = torch.empty(c, 9 * cout, device=dev, dtype=torch.bfloat16)
                job(0, w.data_ptr(), fwd.data_ptr(), n=w.numel())
                for t in range(9):  # bwd[c][t][co] = w[co][8 - t][c] (flipped taps, transposed)
                    job(1, w.data_ptr() + (8 - t) * c * 4, bwd.data_ptr() + t * cout * 2, R=cout, C=c, sld=9 * c,
                        dld=9 * cout)
            self.images.append((fwd, bwd))
        self.items = items
        self.table = torch.tensor(list(b"".join(recs)), dtype=torch.uint8).to(dev)
        self.njobs = len(recs)

    @staticmethod
    def supported(w: torch.Tensor) -> bool:
        if not (w.is_cuda and w.dtype == torch.float32 and w.dim() == 4):
            return False
        cout, c, kh, kw = w.shape
        if (kh, kw) == (1, 1):
            return w.is_contiguous() and cout % 64 == 0 and c % 64 == 0
        return (kh, kw) == (3, 3) and w.is_contiguous(memory_format=torch.channels_last) and cout % 64 == 0 \
            and c % 64 == 0

    def refresh(self) -> None:
        """Rewrite every image from the current weights (one launch) and mark them current."""
        dev = self.weights[0].device
        check(_fns()["run"](ptr(self.table), self.njobs, self.items, stream_handle(dev)), "mifx_weight_prep")
        for w, im in zip(self.weights, self.images):
            _ACTIVE[id(w)] = (w, w._version, im)

    def close(self) -> None:
        for w in self.weights:
            e = _ACTIVE.get(id(w))
            if e is not None and e[0] is w:
                del _ACTIVE[id(w)]
