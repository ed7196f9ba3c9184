"""One-shot gradient exchange over xGMI for the fused W&D data-parallel step (csrc/xgmi.hip, csrc/wide_deep.hip
wd_reduce_xgmi_opt).

One process per GPU. Each rank owns two IPC-exportable device buffers: `part` [2, stride] fp32 (its local
gradient, double-buffered by epoch parity) and `sig` (uncached per-chunk epoch flags, [chunks][8]). The handles
are all-gathered over the trainer's process group once; afterwards a training step needs no host collective:

    fused fwd/bwd  ->  wd_reduce_xgmi_publish: per chunk of columns, reduce the slab, store the chunk into
    part[e & 1], publish epoch e to every peer  ->  wd_xgmi_gather_opt: wait for all peers' e, sum the world
    partials (rank order: bit-identical replicas), optimizer

so the whole data-parallel step is graph-capturable (multi-step hipGraphs like the single-GPU step). The W&D
gradient is one 82 KB bucket: every GPU reads 7 x 82 KB from its peers over 7 point-to-point xGMI links in one
round, where a ring all-reduce pays 2 (N - 1) hop latencies. The reference trains its Wide&Deep with TF
Estimator on one host (airflow-dags/taxi_utils.py:285-356); its distributed path is a
TFJob parameter-server job (notebooks/training-jobs/distributed-tensorflow-training-job.yaml:1-18).

Safety: the wait is a bounded spin (seconds); a peer that never publishes sets `err` instead of hanging the GPU
(`check()` raises). `selftest()` runs the same kernel on a known pattern before the trainer trusts it."""
from __future__ import annotations

import ctypes
import functools

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops._lib import I32, VP, check, ptr, sig, stream_handle

MAX_WORLD = 8


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("xgmi")
    return {
        "hsize": sig(lib, "mifx_xgmi_handle_size", []),
        "malloc": sig(lib, "mifx_xgmi_malloc", [ctypes.c_size_t, I32, ctypes.POINTER(VP)]),
        "free": sig(lib, "mifx_xgmi_free", [VP]),
        "export": sig(lib, "mifx_xgmi_export", [VP, VP]),
        "open": sig(lib, "mifx_xgmi_open", [VP, ctypes.POINTER(VP)]),
        "close": sig(lib, "mifx_xgmi_close", [VP]),
    }


class XgmiExchange:
    """IPC-shared partial/flag buffers of all ranks of `pg` (world 2..8, one GPU each)."""

    def __init__(self, stride: int, pg, device: torch.device):
        from ..ops import wide_deep as wdk

        self.f = _fns()
        self.rank, self.world = dist.get_rank(pg), dist.get_world_size(pg)
        if not 1 <= self.world <= MAX_WORLD:
            raise ValueError(f"xGMI exchange supports 1..{MAX_WORLD} ranks, got {self.world}")
        self.pg, self.device, self.stride = pg, torch.device(device), int(stride)
        self._own, self._opened = [], []
        # Every collective below is reached by every rank whatever fails locally, and failures are agreed on,
        # so all ranks raise together instead of leaving a peer blocked in a collective.
        part, flags, mine, err = VP(), VP(), None, ""
        try:
            with torch.cuda.device(self.device):
                check(self.f["malloc"](2 * self.stride * 4, 0, ctypes.byref(part)), "xgmi malloc(part)")
                self._own.append(part)
                nchunks = wdk._fns()["xgmi_chunks"](self.stride)
                check(self.f["malloc"](nchunks * MAX_WORLD * 4, 1, ctypes.byref(flags)), "xgmi malloc(sig, uncached)")
                self._own.append(flags)
                hs = self.f["hsize"]()
                hp, hf = (ctypes.c_char * hs)(), (ctypes.c_char * hs)()
                check(self.f["export"](part, hp), "hipIpcGetMemHandle(part)")
                check(self.f["export"](flags, hf), "hipIpcGetMemHandle(sig)")
                mine = (bytes(hp), bytes(hf))
        except Exception as e:  # noqa: BLE001 -- reported to all ranks below
            err = f"rank {self.rank}: {e}"
        handles = [None] * self.world
        dist.all_gather_object(handles, (mine, err), group=pg)
        self._agree([e for _, e in handles])
        parts, sigs = [], []
        try:
            with torch.cuda.device(self.device):
                for p, ((a, b), _) in enumerate(handles):
                    if p == self.rank:
                        parts.append(part.value)
                        sigs.append(flags.value)
                        continue
                    pa, pb = VP(), VP()
                    check(self.f["open"](a, ctypes.byref(pa)), f"hipIpcOpenMemHandle(part of rank {p})")
                    self._opened.append(pa)
                    check(self.f["open"](b, ctypes.byref(pb)), f"hipIpcOpenMemHandle(sig of rank {p})")
                    self._opened.append(pb)
                    parts.append(pa.value)
                    sigs.append(pb.value)
        except Exception as e:  # noqa: BLE001
            err = f"rank {self.rank}: {e}"
        errs = [None] * self.world
        dist.all_gather_object(errs, err, group=pg)
        self._agree(errs)
        self.part, self.sig = part, flags
        self.parts = (VP * self.world)(*parts)
        self.sigs = (VP * self.world)(*sigs)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.xctr = torch.zeros(wdk.STEP_SLOTS, dtype=torch.int64, device=self.device)  # epoch slots
        dist.barrier(group=pg)  # every rank's buffers exist and are zeroed before any flag is stored

    def _agree(self, errs) -> None:
        bad = [e for e in errs if e]
        if bad:
            self._release()
            raise RuntimeError("xGMI exchange setup failed: " + "; ".join(bad))

    def _release(self) -> None:
        for p in self._opened:
            self.f["close"](p)
        self._opened = []
        for p in self._own:
            self.f["free"](p)
        self._own = []

    # ------------------------------------------------------------------ step (stream ordered)
    def reduce_apply(self, tr) -> None:
        """Slab reduction + exchange + optimizer of FusedWideDeepTrainer `tr`: local sum (XCD-local when the trainer
        has the XcdReduce scratch and the kernel recorded workgroup XCDs) published to the peers, then gather +
        optimizer."""
        from ..ops import wide_deep as wdk

        xr = getattr(tr, "_xcd", None)
        if xr is not None and getattr(xr, "xcd_of", None) is None:
            xr = None  # (a reduction scratch without a placement record: the kernel's one-pass local sum)
        xa = (ptr(xr.xcd_of), ptr(xr.part), ptr(xr.ok), ptr(xr.xep)) if xr is not None else (None,) * 4
        rc = wdk._fns()["reduce_xgmi_opt"](ptr(tr.slab), int(tr.grid), self.stride, self.parts, self.sigs, self.world,
                                           self.rank, self.sig, ptr(self.err), ptr(self.xctr), None, ptr(tr.wsc),
                                           ptr(tr.param_sc), ptr(tr.s0_sc), ptr(tr.s1_sc), ptr(tr.wt),
                                           ptr(tr.step_ctr), ptr(tr.h_dnn), ptr(tr.h_wide), *xa,
                                           stream_handle(self.device))
        check(rc, "mifx_wd_reduce_xgmi_opt")

    def sum_into(self, slab: torch.Tensor, out: torch.Tensor) -> None:
        """Plain exchange (no optimizer): out[stride] = sum over ranks of each rank's slab row sum."""
        from ..ops import wide_deep as wdk

        rc = wdk._fns()["reduce_xgmi_opt"](ptr(slab), int(slab.shape[0]), self.stride, self.parts, self.sigs,
                                           self.world, self.rank, self.sig, ptr(self.err), ptr(self.xctr), ptr(out),
                                           None, None, None, None, None, None, None, None, None, None, None, None,
                                           stream_handle(self.device))
        check(rc, "mifx_wd_reduce_xgmi_opt(sum)")

    # ------------------------------------------------------------------ validation
    def check(self) -> None:
        if int(self.err.item()) != 0:
            raise RuntimeError("xGMI exchange: a peer never published its epoch (wait timed out)")

    def selftest(self) -> None:
        """Exchange a known pattern through the real kernel and compare with the exact sum (all ranks)."""
        try:
            with torch.cuda.device(self.device):
                i = torch.arange(self.stride, device=self.device, dtype=torch.float32)
                mine = (self.rank + 1) * (torch.remainder(i, 97) + 1) * 0.5  # exact in fp32
                want = (self.world * (self.world + 1) // 2) * (torch.remainder(i, 97) + 1) * 0.5
                out = torch.empty(self.stride, device=self.device)
                self.sum_into(mine.view(1, -1), out)
                torch.cuda.synchronize(self.device)
                self.check()
                ok = torch.equal(out, want)
        except Exception:  # noqa: BLE001 -- agreed on below, every rank reaches the all-reduce
            ok = False
        fdev = self.device if dist.get_backend(self.pg) == "nccl" else torch.device("cpu")
        flag = torch.tensor([0 if ok else 1], dtype=torch.int64, device=fdev)
        dist.all_reduce(flag, group=self.pg)  # every rank learns whether any rank saw a wrong sum
        if not ok or int(flag.item()) != 0:
            raise RuntimeError("xGMI exchange self-test: wrong sum")

    def close(self) -> None:
        """Collective: unmap the peers' buffers and free ours once nobody reads them."""
        if not self._own:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.pg)  # nobody reads our buffers any more
        for p in self._opened:
            self.f["close"](p)
        self._opened = []
        dist.barrier(group=self.pg)
        self._release()
