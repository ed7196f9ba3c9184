"""ctypes bindings for csrc/wd_chain.hip (register-chained fused Wide&Deep step on gfx950)."""
from __future__ import annotations

import ctypes
import functools

import torch

from . import _lib
from ._lib import F32, I32, I64, U64, VP, check, ptr, sig, stream_handle


# mifx_wdc_fused_help: records, n_data, batch, step slots, image, wide, slab, slab_loss, grad_scale, tile map, stride,
# bar, err, wsc, param, s0, s1, hyper dnn / wide, helpers, feed stride / offset / key, stream
HELP_SIG = [VP, I64, I64, VP, VP, VP, VP, VP, F32, VP, I32, VP, VP, VP, VP, VP, VP, VP, VP, I32, I64, I64, U64, VP]


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("wd_chain")
    return {
        "constants": sig(lib, "mifx_wdc_constants", [VP, I32]),
        "fused": sig(lib, "mifx_wdc_fused", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP, I32, I32,
                                             VP]),
        "fused_x": sig(lib, "mifx_wdc_fused_x", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP, I32,
                                                 I32, VP, VP]),
        "fused_f": sig(lib, "mifx_wdc_fused_f", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP, I32,
                                                 I32, VP, I64, I64, U64, VP]),
        "fused_tail": sig(lib, "mifx_wdc_fused_tail", [VP, I64, I64, VP, VP, VP, VP, VP, F32, I32, VP, I32, VP, VP, VP,
                                                       VP, VP, VP, VP, VP, VP, VP, VP, I64, I64, U64, VP]),
        "persist": sig(lib, "mifx_wdc_persist", [VP, I64, I64, VP, VP, VP, VP, VP, F32, VP, I32, VP, VP, VP, VP, VP, VP,
                                                 I32, I64, I64, U64, VP]),
        "help": sig(lib, "mifx_wdc_fused_help", HELP_SIG),
    }


@functools.lru_cache(maxsize=None)
def _fns64():
    """csrc/wd_chain64.hip: the same kernel at 64 examples per iteration (4 waves x 16), the small-batch shape."""
    lib = _lib.load("wd_chain64")
    return {
        "constants": sig(lib, "mifx_wdc_constants_t64", [VP, I32]),
        "fused": sig(lib, "mifx_wdc_fused_t64", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP, I32,
                                                 I32, VP]),
        "fused_x": sig(lib, "mifx_wdc_fused_x_t64", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP,
                                                     I32, I32, VP, VP]),
        "fused_f": sig(lib, "mifx_wdc_fused_f_t64", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP,
                                                     I32, I32, VP, I64, I64, U64, VP]),
        "help": sig(lib, "mifx_wdc_fused_help_t64", HELP_SIG),
    }


@functools.lru_cache(maxsize=None)
def _fns256():
    """csrc/wd_chain256.hip: 256 examples per iteration (8 waves x 32), ONE iteration per workgroup (grid * 256 >=
    batch), layers 1-3 staged in two passes: the large-batch shape."""
    lib = _lib.load("wd_chain256")
    return {
        "constants": sig(lib, "mifx_wdc_constants_t256", [VP, I32]),
        "fused_f": sig(lib, "mifx_wdc_fused_f_t256", [VP, I64, I64, I64, VP, VP, VP, VP, VP, VP, F32, I32, I32, VP,
                                                      I32, I32, VP, I64, I64, U64, VP]),
    }


def fns_for(tile: int) -> dict:
    """Bindings of the T = tile build (128: csrc/wd_chain.hip, 64: csrc/wd_chain64.hip, 256: csrc/wd_chain256.hip)."""
    if tile not in (64, 128, 256):
        raise ValueError("tile must be 64, 128 or 256")
    return {128: _fns, 64: _fns64, 256: _fns256}[tile]()


@functools.lru_cache(maxsize=None)
def constants() -> dict[str, int]:
    buf = (ctypes.c_int * 16)()
    n = _fns()["constants"](buf, 16)
    names = ["T", "LWEND", "LDS_BYTES", "PAD", "NTILE", "WIDE_PAD", "LW1", "LW2", "LW3", "LW4", "LW5"]
    return {k: buf[i] for i, k in enumerate(names[:n])}


def fused(records: torch.Tensor, n_data: int, batch: int, start_fixed: int, step_ctr: torch.Tensor | None,
          wimg_bf16: torch.Tensor, wide: torch.Tensor, slab: torch.Tensor | None, slab_loss: torch.Tensor | None,
          logits_out: torch.Tensor | None, grad_scale: float, grid: int, train: bool,
          tmap: torch.Tensor | None = None, waves: int = 8, xcd_of: torch.Tensor | None = None,
          tile: int = 128, feed: tuple[int, int, int] | None = None) -> None:
    """One chained-kernel launch. wimg_bf16: [LWEND] bf16 (or int16) weight image in the kernel's LDS layout
    (models.wide_deep.chain_image); slab: [>= grid, stride] with the chain_maps() compact layout.
    tile 128: waves 8 (two waves per SIMD, 16 examples each) or 4 (one wave per SIMD, 32 examples each);
    tile 64 (64 examples per workgroup iteration): waves 4 (one wave per SIMD, 16 examples each). xcd_of: int32
    [>= grid], receives the XCD each workgroup ran on (for the XCD-local slab reduction). feed: (stride, offset,
    shuffle seed) of the record stream (csrc/feed.h, mifx.data.shuffle); None = (batch, 0, 0), stored order."""
    if waves not in {128: (4, 8), 64: (4,), 256: (8,)}[tile]:
        raise ValueError("waves must be 4 or 8 (tile 128) / 4 (tile 64) / 8 (tile 256)")
    if tile == 256 and train and grid * 256 < batch:
        raise ValueError("tile 256 runs one iteration per workgroup: grid * 256 >= batch")
    c = constants()
    if wimg_bf16.numel() != c["LWEND"] or wimg_bf16.element_size() != 2 or not wimg_bf16.is_contiguous():
        raise ValueError("weight image must be a contiguous 16-bit [LWEND] tensor")
    if records.dim() != 2 or records.shape[1] != 32 or not records.is_contiguous():
        raise ValueError("records must be contiguous uint8 [N, 32]")
    stride = int(slab.shape[-1]) if slab is not None else 0
    if train:
        if tmap is None or tmap.dtype != torch.int32 or tmap.numel() != c["NTILE"]:
            raise ValueError("training launch needs the int32 tile map of the chained slab layout")
        if slab.shape[0] < grid or not slab.is_contiguous():
            raise ValueError("slab must be a contiguous [>= grid, stride] tensor")
        if slab_loss is not None and slab_loss.numel() < grid:
            raise ValueError("slab_loss must hold >= grid floats")
    elif logits_out is None or logits_out.numel() < batch:
        raise ValueError("eval launch needs logits_out with >= batch floats")
    if xcd_of is not None and (xcd_of.dtype != torch.int32 or xcd_of.numel() < grid):
        raise ValueError("xcd_of must be int32 [>= grid]")
    gs, go, key = feed if feed is not None else (batch, 0, 0)
    rc = fns_for(tile)["fused_f"](ptr(records), n_data, batch, start_fixed, ptr(step_ctr), ptr(wimg_bf16), ptr(wide),
                                  ptr(slab), ptr(slab_loss), ptr(logits_out), float(grad_scale), int(grid), int(train),
                                  ptr(tmap), stride, int(waves), ptr(xcd_of), int(gs), int(go), int(key) & (2**64 - 1),
                                  stream_handle(records.device))
    check(rc, "mifx_wdc_fused")


class InKernelTail:
    """Scratch of the one-launch training step (csrc/wd_chain.hip TailArgs): the slab reduction and the optimizer
    run inside the fused kernel after two grid-wide barriers. xcd_of [256], per-XCD partials [16, stride], the
    monotonic barrier counter and the sticky error flag (set when a barrier wait timed out: the step then skipped
    its update; `check()` raises)."""

    def __init__(self, stride: int, device):
        self.stride = int(stride)
        self.xcd_of = torch.zeros(256, dtype=torch.int32, device=device)
        self.xpart = torch.zeros(16 * self.stride, device=device)
        self.bar = torch.zeros(1, dtype=torch.int64, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.dbg = None  # [256, 8] int64 real-time stamps when set (tools/tail_stamps.py)

    def step(self, tr) -> None:
        """One training step of FusedWideDeepTrainer `tr` (chained kernel, slab-column-order state)."""
        c = constants()
        if tr.wt.numel() != c["LWEND"] or tr.tmap.numel() != c["NTILE"] or tr.slab.shape[0] < tr.grid:
            raise ValueError("trainer buffers do not match the chained kernel")
        if tr.grid > 256 or tr.stride != self.stride:
            raise ValueError("in-kernel tail: grid <= 256 and the trainer's slab stride")
        rc = _fns()["fused_tail"](ptr(tr.records), tr.n_data, tr.batch, ptr(tr.step_ctr), ptr(tr.wt),
                                  ptr(tr.wide_weights), ptr(tr.slab), ptr(tr.slab_loss), float(tr.grad_scale),
                                  int(tr.grid), ptr(tr.tmap), int(tr.stride), ptr(self.xcd_of), ptr(self.xpart),
                                  ptr(self.bar), ptr(self.err), ptr(tr.wsc), ptr(tr.param_sc), ptr(tr.s0_sc),
                                  ptr(tr.s1_sc), ptr(tr.h_dnn), ptr(tr.h_wide), ptr(self.dbg), *tr.feed_args(),
                                  stream_handle(tr.records.device))
        check(rc, "mifx_wdc_fused_tail")

    def check(self) -> None:
        if int(self.err.item()) != 0:
            raise RuntimeError("W&D in-kernel tail: a grid barrier timed out (workgroups not co-resident); the "
                               "step skipped its update")


class OneRowTail:
    """One launch per step for a batch ONE workgroup trains (csrc/wd_chain.hip help_update): workgroup 0 runs the
    fused step, `helpers` more workgroups run the optimizer over the slab columns (wd_opt1_sc's partition: one thread
    per column, step slot per workgroup), loading their state during the step and updating once workgroup 0 has
    published the gradient row. `bar` holds the last published step (reset whenever the step slots are rewritten);
    `err` is the sticky timeout flag (`check()` raises)."""

    def __init__(self, stride: int, tile: int, device):
        self.stride, self.tile = int(stride), int(tile)
        threads = 256 if self.tile == 64 else 512
        self.helpers = -(-self.stride // threads)
        self.bar = torch.empty(1, dtype=torch.int64, device=device)
        self.err = torch.zeros(1, dtype=torch.int32, device=device)
        self.reset()

    def reset(self) -> None:
        self.bar.fill_(-1)  # matches no step

    def step(self, tr) -> None:
        c = constants()
        if tr.wt.numel() != c["LWEND"] or tr.tmap.numel() != c["NTILE"] or tr.stride != self.stride:
            raise ValueError("trainer buffers do not match the chained kernel")
        rc = fns_for(self.tile)["help"](ptr(tr.records), tr.n_data, tr.batch, ptr(tr.step_ctr), ptr(tr.wt),
                                        ptr(tr.wide_weights), ptr(tr.slab), ptr(tr.slab_loss), float(tr.grad_scale),
                                        ptr(tr.tmap), int(tr.stride), ptr(self.bar), ptr(self.err), ptr(tr.wsc),
                                        ptr(tr.param_sc), ptr(tr.s0_sc), ptr(tr.s1_sc), ptr(tr.h_dnn), ptr(tr.h_wide),
                                        int(self.helpers), *tr.feed_args(), stream_handle(tr.records.device))
        check(rc, "mifx_wdc_fused_help")

    def check(self) -> None:
        if int(self.err.item()) != 0:
            raise RuntimeError("W&D one-launch step: the optimizer workgroups timed out waiting for the gradient row; "
                               "the step skipped its update")


def persist_steps(tr, nsteps: int) -> None:
    """`nsteps` training steps of FusedWideDeepTrainer `tr` (chained kernel, one rank, batch <= T) in ONE launch of
    the persistent single-workgroup kernel (csrc/wd_chain.hip opt_tiles / mifx_wdc_persist): the weight image stays
    in LDS across the steps and the optimizer runs inside the workgroup."""
    c = constants()
    if tr.wt.numel() != c["LWEND"] or tr.tmap.numel() != c["NTILE"]:
        raise ValueError("trainer buffers do not match the chained kernel")
    if tr.batch > c["T"] or nsteps <= 0:
        raise ValueError(f"persistent step: batch <= {c['T']} and nsteps >= 1")
    rc = _fns()["persist"](ptr(tr.records), tr.n_data, tr.batch, ptr(tr.step_ctr), ptr(tr.wt), ptr(tr.wide_weights),
                           ptr(tr.slab), ptr(tr.slab_loss), float(tr.grad_scale), ptr(tr.tmap), int(tr.stride), ptr(tr.wsc),
                           ptr(tr.param_sc), ptr(tr.s0_sc), ptr(tr.s1_sc), ptr(tr.h_dnn), ptr(tr.h_wide),
                           int(nsteps), *tr.feed_args(), stream_handle(tr.records.device))
    check(rc, "mifx_wdc_persist")
