"""ctypes bindings for csrc/wide_deep.hip (fused Wide&Deep train/eval step on gfx950)."""
from __future__ import annotations

import ctypes
import functools
import os

import torch

from . import _lib
from ._lib import F32, I32, I64, U64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("wide_deep")
    return {
        "constants": sig(lib, "mifx_wd_constants", [VP, I32]),
        "fused": sig(lib, "mifx_wd_fused", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP, I32, VP,
                                            I64, I64, U64, VP]),
        "reduce": sig(lib, "mifx_wd_reduce", [VP, I32, I32, VP, I32, VP]),
        "optimizer": sig(lib, "mifx_wd_optimizer", [VP, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP, I32, VP]),
        "reduce_opt": sig(lib, "mifx_wd_reduce_opt", [VP, I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
        "reduce_opt_sc": sig(lib, "mifx_wd_reduce_opt_sc", [VP, I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
        "xcd_chunks": sig(lib, "mifx_wd_xcd_chunks", [I32]),
        "reduce_xcd_opt": sig(lib, "mifx_wd_reduce_xcd_opt", [VP, I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP,
                                                              VP, VP, VP, VP]),
        "reduce_res_opt": sig(lib, "mifx_wd_reduce_res_opt", [VP, I32, I32, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP,
                                                              VP]),
        "reduce_res_opt_fused": sig(lib, "mifx_wd_reduce_res_opt_fused", [VP, I32, I32, VP, VP, VP, VP, VP, VP, VP,
                                                                          VP, VP, VP, VP]),
        "xgmi_chunks": sig(lib, "mifx_wd_xgmi_chunks", [I32]),
        "reduce_xgmi_opt": sig(lib, "mifx_wd_reduce_xgmi_opt", [VP, I32, I32, VP, VP, I32, I32, VP, VP, VP, VP, VP,
                                                                VP, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
    }


@functools.lru_cache(maxsize=None)
def constants() -> dict[str, int]:
    buf = (ctypes.c_int * 32)()
    n = _fns()["constants"](buf, 32)
    names = ["T", "WTOT", "NWIDE", "STRIDE", "NTILE", "LDS_BYTES", "OFF1", "OFF2", "OFF3", "OFF4", "OFF5",
             "TB1", "TB2", "TB3", "TB4", "TB5"]
    return {k: buf[i] for i, k in enumerate(names[:n])}


def fused(records: torch.Tensor, n_data: int, batch: int, start_fixed: int, step_ctr: torch.Tensor | None,
          wt_bf16: torch.Tensor, wide: torch.Tensor, slab: torch.Tensor | None, slab_loss: torch.Tensor | None,
          logits_out: torch.Tensor | None, grad_scale: float, grid: int, train: bool,
          tmap: torch.Tensor | None = None, stage_dims=None, feed: tuple[int, int, int] | None = None) -> None:
    """slab: [grid, stride] with stride = slab.shape[1] (compact layout of `tmap`, see
    models.wide_deep.compact_tile_map). stage_dims: 10 ints (live rows[5], 16-B granules per row[5]) of
    the weight image to stage (models.wide_deep.stage_dims); None stages the whole padded image. feed: (stride,
    offset, shuffle seed) of the record stream (csrc/feed.h); None = (batch, 0, 0), stored order."""
    sd = None
    if stage_dims is not None:
        sd = (ctypes.c_int * 10)(*[int(v) for v in stage_dims])
    stride = int(slab.shape[-1]) if slab is not None else 0
    if train:
        if tmap is None or tmap.dtype != torch.int32 or tmap.numel() != constants()["NTILE"]:
            raise ValueError("training launch needs the int32 tile map of the compact slab layout")
        if slab.shape[0] < grid or not slab.is_contiguous():
            raise ValueError("slab must be a contiguous [>= grid, stride] tensor")
    rc = _fns()["fused"](ptr(records), n_data, batch, start_fixed, ptr(step_ctr), ptr(wt_bf16), ptr(wide), ptr(slab),
                         ptr(slab_loss), ptr(logits_out), float(grad_scale), int(grid), int(train), ptr(tmap), stride,
                         sd, *(feed_args(feed, batch)), stream_handle(records.device))
    check(rc, "mifx_wd_fused")


def feed_args(feed, batch: int) -> tuple[int, int, int]:
    gs, go, key = feed if feed is not None else (batch, 0, 0)
    return int(gs), int(go), int(key) & (2**64 - 1)


def reduce(slab: torch.Tensor, groups: int, nsplit: int, partial: torch.Tensor) -> None:
    if partial.shape[-1] != slab.shape[-1] or partial.numel() < nsplit * slab.shape[-1]:
        raise ValueError("partial must be [>= nsplit, stride] with the slab's stride")
    check(_fns()["reduce"](ptr(slab), groups, nsplit, ptr(partial), int(slab.shape[-1]), stream_handle(slab.device)),
          "mifx_wd_reduce")


STEP_SLOTS = 512  # csrc/wide_deep.hip: one step slot per optimizer workgroup, slot 0 = canonical step


def _check_step_ctr(step_ctr: torch.Tensor) -> None:
    if step_ctr.dtype != torch.int64 or step_ctr.numel() < STEP_SLOTS or not step_ctr.is_contiguous():
        raise ValueError(f"step_ctr must be a contiguous int64 tensor of {STEP_SLOTS} per-workgroup step slots")


def reduce_full(slab: torch.Tensor, groups: int, out: torch.Tensor) -> None:
    """out[stride] = sum of the first `groups` slab rows (one launch, fixed summation order)."""
    stride = int(slab.shape[-1])
    if out.numel() < stride or slab.numel() < groups * stride or not slab.is_contiguous():
        raise ValueError("slab must be contiguous [>= groups, stride] and out hold >= stride floats")
    rc = _fns()["reduce_opt"](ptr(slab), int(groups), stride, ptr(out), None, None, None, None, None, None, None,
                              None, None, stream_handle(slab.device))
    check(rc, "mifx_wd_reduce_opt")


def reduce_apply(slab: torch.Tensor, groups: int, inv: torch.Tensor, param: torch.Tensor, s0: torch.Tensor,
                 s1: torch.Tensor, wt_out: torch.Tensor, step_ctr: torch.Tensor, hyper_dnn: torch.Tensor,
                 hyper_wide: torch.Tensor, wmap: torch.Tensor | None = None) -> None:
    """Sum the first `groups` slab rows and apply the optimizer in the same launch. inv: int32 [stride]
    slab column -> canonical parameter index (-1 for padding), see FusedWideDeepTrainer. wmap: int32 [WTOT]
    canonical DNN index -> offset in wt_out (the register-chained kernel's C-ordered image); None writes
    wt_out in canonical order."""
    if wmap is not None and (wmap.dtype != torch.int32 or wmap.numel() < param.numel() - 2128):
        raise ValueError("wmap must be int32 [WTOT]")
    stride = int(slab.shape[-1])
    if inv.dtype != torch.int32 or inv.numel() != stride:
        raise ValueError("inv must be int32 [stride]")
    if slab.numel() < groups * stride or not slab.is_contiguous():
        raise ValueError("slab must be contiguous [>= groups, stride]")
    _check_step_ctr(step_ctr)
    rc = _fns()["reduce_opt"](ptr(slab), int(groups), stride, None, ptr(inv), ptr(param), ptr(s0), ptr(s1),
                              ptr(wt_out), ptr(wmap), ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide),
                              stream_handle(param.device))
    check(rc, "mifx_wd_reduce_opt")


def reduce_apply_sc(slab: torch.Tensor, groups: int, wsc: torch.Tensor, param_sc: torch.Tensor, s0_sc: torch.Tensor,
                    s1_sc: torch.Tensor, wt_out: torch.Tensor, step_ctr: torch.Tensor, hyper_dnn: torch.Tensor,
                    hyper_wide: torch.Tensor) -> None:
    """Slab [groups, stride] -> sum -> optimizer on slab-column-order state (csrc/wide_deep.hip wd_reduce_opt_sc)."""
    stride = slab.shape[-1]
    for t in (wsc, param_sc, s0_sc, s1_sc):
        if t.numel() != stride or not t.is_contiguous():
            raise ValueError("slab-order state must be contiguous [stride]")
    _check_step_ctr(step_ctr)
    rc = _fns()["reduce_opt_sc"](ptr(slab), int(groups), stride, ptr(wsc), ptr(param_sc), ptr(s0_sc), ptr(s1_sc),
                                 ptr(wt_out), ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide),
                                 stream_handle(param_sc.device))
    check(rc, "mifx_wd_reduce_opt_sc")


class XcdReduce:
    """Scratch for the XCD-local two-level slab reduction + optimizer (csrc/wide_deep.hip wd_reduce_xcd /
    wd_xcd_opt_sc): xcd_of [256] (filled by the chained kernel), per-XCD partials [16, stride], epoch stamps and
    epoch slots."""

    def __init__(self, stride: int, device):
        nc1 = _fns()["xcd_chunks"](int(stride))
        self.stride = int(stride)
        self.xcd_of = torch.zeros(256, dtype=torch.int32, device=device)
        self.part = torch.zeros(16 * stride, device=device)
        self.ok = torch.zeros(16 * nc1, dtype=torch.int32, device=device)
        self.xep = torch.zeros(STEP_SLOTS, dtype=torch.int64, device=device)

    def _call(self, slab, groups, out, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn, hyper_wide):
        rc = _fns()["reduce_xcd_opt"](ptr(slab), int(groups), self.stride, ptr(self.xcd_of), ptr(self.part),
                                      ptr(self.ok), ptr(self.xep), ptr(out), ptr(wsc), ptr(param_sc), ptr(s0_sc),
                                      ptr(s1_sc), ptr(wt_out), ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide),
                                      stream_handle(slab.device))
        check(rc, "mifx_wd_reduce_xcd_opt")

    def apply_sc(self, slab: torch.Tensor, groups: int, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn,
                 hyper_wide) -> None:
        _check_step_ctr(step_ctr)
        if self.fused:
            if slab.shape[-1] != self.stride or slab.numel() < groups * self.stride or not slab.is_contiguous():
                raise ValueError("slab must be contiguous [>= groups, stride]")
            rc = _fns()["reduce_res_opt_fused"](ptr(slab), int(groups), self.stride, ptr(self.part), ptr(self.ticket),
                                                ptr(wsc), ptr(param_sc), ptr(s0_sc), ptr(s1_sc), ptr(wt_out),
                                                ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide),
                                                stream_handle(slab.device))
            check(rc, "mifx_wd_reduce_res_opt_fused")
            return
        self._call(slab, groups, None, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn, hyper_wide)

    def sum_into(self, slab: torch.Tensor, groups: int, out: torch.Tensor) -> None:
        self._call(slab, groups, out, None, None, None, None, None, None, None, None)


class ResReduce:
    """Scratch of the residue-class two-level slab reduction + optimizer (csrc/wide_deep.hip wd_reduce_res /
    wd_res_opt_sc): per-residue partials [8, stride]. Same interface as XcdReduce."""

    def __init__(self, stride: int, device, fused: bool | None = None):
        self.stride = int(stride)
        self.part = torch.zeros(8 * stride, device=device)
        self.xcd_of = None  # (no placement record needed)
        # fused (MIFX_WD_RES_FUSED=1): both levels in one launch, the optimizer run by the last of a chunk's residue
        # workgroups (csrc/wide_deep.hip wd_reduce_res_fused); per-chunk tickets, zero between calls. Bit-identical
        # to the two launches but measured slower on the headline step: 29.7-29.9 vs 28.3-28.5 us (release-fenced
        # ticket: 33.4-33.6), profiles/wd_res_fused_ab_r6.jsonl -- opt-in
        self.fused = os.environ.get("MIFX_WD_RES_FUSED", "0") == "1" if fused is None else bool(fused)
        self.ticket = torch.zeros((self.stride + 255) // 256, dtype=torch.int32, device=device)

    def _call(self, slab, groups, out, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn, hyper_wide):
        if slab.shape[-1] != self.stride or slab.numel() < groups * self.stride or not slab.is_contiguous():
            raise ValueError("slab must be contiguous [>= groups, stride]")
        rc = _fns()["reduce_res_opt"](ptr(slab), int(groups), self.stride, ptr(self.part), ptr(out), ptr(wsc),
                                      ptr(param_sc), ptr(s0_sc), ptr(s1_sc), ptr(wt_out), ptr(step_ctr),
                                      ptr(hyper_dnn), ptr(hyper_wide), stream_handle(slab.device))
        check(rc, "mifx_wd_reduce_res_opt")

    def apply_sc(self, slab: torch.Tensor, groups: int, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn,
                 hyper_wide) -> None:
        _check_step_ctr(step_ctr)
        if self.fused:
            if slab.shape[-1] != self.stride or slab.numel() < groups * self.stride or not slab.is_contiguous():
                raise ValueError("slab must be contiguous [>= groups, stride]")
            rc = _fns()["reduce_res_opt_fused"](ptr(slab), int(groups), self.stride, ptr(self.part), ptr(self.ticket),
                                                ptr(wsc), ptr(param_sc), ptr(s0_sc), ptr(s1_sc), ptr(wt_out),
                                                ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide),
                                                stream_handle(slab.device))
            check(rc, "mifx_wd_reduce_res_opt_fused")
            return
        self._call(slab, groups, None, wsc, param_sc, s0_sc, s1_sc, wt_out, step_ctr, hyper_dnn, hyper_wide)

    def sum_into(self, slab: torch.Tensor, groups: int, out: torch.Tensor) -> None:
        self._call(slab, groups, out, None, None, None, None, None, None, None, None)


def optimizer(partial: torch.Tensor, nparts: int, gidx: torch.Tensor, mask: torch.Tensor, param: torch.Tensor,
              s0: torch.Tensor, s1: torch.Tensor, wt_out: torch.Tensor, step_ctr: torch.Tensor,
              hyper_dnn: torch.Tensor, hyper_wide: torch.Tensor) -> None:
    # hyper tensors live on the host (read by the launcher, passed by value)
    _check_step_ctr(step_ctr)
    rc = _fns()["optimizer"](ptr(partial), nparts, ptr(gidx), ptr(mask), ptr(param), ptr(s0), ptr(s1), ptr(wt_out),
                             ptr(step_ctr), ptr(hyper_dnn), ptr(hyper_wide), int(partial.shape[-1]),
                             stream_handle(param.device))
    check(rc, "mifx_wd_optimizer")
