"""Fused BatchNorm + ReLU over channels_last activations (csrc/bn_relu.hip).

`BatchNormReLU2d` is a drop-in `nn.BatchNorm2d` (same parameters, buffers and state_dict keys)
whose forward is relu(batch_norm(x)). On the GPU with a channels_last (NHWC) bf16/fp32 input and
C % 8 == 0 it runs the native kernels — training: stats -> finalize (running stats updated on the
device) -> apply; backward: reduce -> finalize -> apply — and fails loudly if the library is
missing. Elsewhere (CPU, other layouts) it runs the PyTorch reference of the same math."""
from __future__ import annotations

import functools

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("bn_relu")
    return {
        "blocks": sig(lib, "mifx_bn_blocks", [I64, I32]),
        "fwd": sig(lib, "mifx_bn_relu_fwd",
                   [I32, VP, VP, VP, I64, I32, VP, VP, F32, F32, VP, VP, I32, VP, VP, VP, VP]),
        "apply": sig(lib, "mifx_bn_relu_apply", [I32, VP, I64, I32, VP, VP, I32, VP, VP]),
        "bwd": sig(lib, "mifx_bn_relu_bwd", [I32, VP, VP, VP, I64, I32, VP, VP, I32, VP, VP, VP, VP, VP, VP]),
        "fwd_tiles": sig(lib, "mifx_bn_relu_fwd_tiles",
                         [I32, VP, I64, I32, VP, I32, I32, VP, VP, F32, F32, VP, VP, I32, VP, VP, VP, VP]),
        "tiles_ws": sig(lib, "mifx_bn_tiles_ws", [I32, I32]),
        "bwd_tiles": sig(lib, "mifx_bn_relu_bwd_tiles",
                         [I32, VP, VP, VP, I64, I32, VP, VP, I32, VP, VP, I32, VP, VP, VP, VP, VP, VP]),
    }


def _nhwc_view(x: torch.Tensor) -> torch.Tensor | None:
    """[N, C, H, W] channels_last (or [M, C] row-major) -> the [M, C] storage view, else None."""
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = x.shape
        return x.permute(0, 2, 3, 1).reshape(n * h * w, c)
    if x.dim() == 2 and x.is_contiguous():
        return x
    return None


def native_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    v = _nhwc_view(x)
    c = x.shape[1]
    return v is not None and c % 8 == 0 and c <= 2048 and x.data_ptr() % 16 == 0 and v.shape[0] > 0


def _dt(t: torch.Tensor) -> int:
    return 1 if t.dtype == torch.bfloat16 else 0


def _fwd(x, x2, weight, bias, run_mean, run_var, momentum, eps, relu):
    """Launch the fused forward; returns (y, s, w32, stats) where s = x + x2 (or x when x2 is None)."""
    v = _nhwc_view(x)
    M, C = v.shape
    w32, b32 = weight.float().contiguous(), bias.float().contiguous()
    nb = _fns()["blocks"](M, C)
    part = torch.empty(2, nb, C, device=x.device, dtype=torch.float32)
    stats = torch.empty(4, C, device=x.device, dtype=torch.float32)
    y = torch.empty_like(x)  # same (channels_last) layout
    s = torch.empty_like(x) if x2 is not None else x
    v2 = _nhwc_view(x2) if x2 is not None else None
    sv = _nhwc_view(s) if x2 is not None else None
    check(_fns()["fwd"](_dt(x), ptr(v), ptr(v2), ptr(sv), M, C, ptr(w32), ptr(b32), float(eps), float(momentum),
                        ptr(run_mean), ptr(run_var if run_mean is not None else None), int(relu), ptr(part),
                        ptr(stats), ptr(y), stream_handle(x.device)), "mifx_bn_relu_fwd")
    return y, s, w32, stats


_LAYOUT_DIAG = __import__("os").environ.get("MIFX_BN_LAYOUT_DIAG") == "1"


def _grad_dests(ctx):
    """(dgamma, dbeta) output tensors: the data-parallel bucket views when the deferred-gradient context hands them out
    (mifx.ops.gemm.grad_destination), else fresh [2, C] fp32 rows."""
    wb = getattr(ctx, "mifx_wb", None)
    if wb is None:
        return None
    from .gemm import grad_destination

    dw, db = (grad_destination(t) for t in wb)
    return (dw, db) if dw is not None and db is not None else None


def _dgb(C, dev, dst):
    if dst is not None:
        return dst
    d = torch.empty(2, C, device=dev, dtype=torch.float32)
    return d[0], d[1]


def _bwd(dy, x, w32, stats, relu, dres, dst=None):
    if _LAYOUT_DIAG:
        for nm, t in (("dy", dy), ("dres", dres)):
            if t is not None and t.dim() == 4 and not t.is_contiguous(memory_format=torch.channels_last):
                print(f"[bn-layout] {nm} {tuple(t.shape)} strides {t.stride()} dtype {t.dtype}", flush=True)
    if dy.dim() == 4 and not dy.is_contiguous(memory_format=torch.channels_last):
        dy = dy.contiguous(memory_format=torch.channels_last)
    dy = dy.to(x.dtype)
    if dres is not None:
        if dres.dim() == 4 and not dres.is_contiguous(memory_format=torch.channels_last):
            dres = dres.contiguous(memory_format=torch.channels_last)
        dres = dres.to(x.dtype)
    v, dv = _nhwc_view(x), _nhwc_view(dy)
    M, C = v.shape
    nb = _fns()["blocks"](M, C)
    part = torch.empty(2, nb, C, device=x.device, dtype=torch.float32)
    kbuf = torch.empty(3, C, device=x.device, dtype=torch.float32)
    dgb = _dgb(C, x.device, dst)
    dx = torch.empty_like(x)
    check(_fns()["bwd"](_dt(x), ptr(dv), ptr(v), ptr(_nhwc_view(dres) if dres is not None else None), M, C, ptr(w32),
                        ptr(stats), int(relu), ptr(part), ptr(kbuf), ptr(dx), ptr(dgb[0]), ptr(dgb[1]),
                        stream_handle(x.device)), "mifx_bn_relu_bwd")
    return dx, dgb


def offer_bwd_tiles(node, dy: torch.Tensor, part: torch.Tensor) -> None:
    """Hand a BatchNorm + ReLU node (the grad_fn of its output) the per-tile backward sums (part: [2, T, C] = sum g,
    sum g xhat) that the GEMM producing its output gradient `dy` reduced in its epilogue (mifx.ops.conv1x1). The node
    uses them only if the gradient it then receives IS dy, unmodified (same storage, same version: no other consumer's
    gradient was accumulated into it), else it runs its own reduction."""
    node.mifx_bwd_tiles = (part, dy.data_ptr(), dy._version)


def _take_tiles(ctx, dy):
    t = getattr(ctx, "mifx_bwd_tiles", None)
    if t is None:
        return None
    ctx.mifx_bwd_tiles = None
    part, p, ver = t
    if dy is None or dy.data_ptr() != p or dy._version != ver or dy.dtype != torch.bfloat16:
        return None
    return part


def _bwd_tiles(dy, x, w32, stats, dres, part, act=None, dst=None):
    """Backward of relu(bn(x)) from the per-tile sums the producing GEMM reduced: finalize + apply only. act: also
    write the forward's activation relu(bn(x)) there (same layout as x)."""
    if dres is not None:
        if dres.dim() == 4 and not dres.is_contiguous(memory_format=torch.channels_last):
            dres = dres.contiguous(memory_format=torch.channels_last)
        dres = dres.to(x.dtype)
    v, dv = _nhwc_view(x), _nhwc_view(dy)
    M, C = v.shape
    T = part.shape[1]
    kbuf = torch.empty(3, C, device=x.device, dtype=torch.float32)
    dgb = _dgb(C, x.device, dst)
    dx = torch.empty_like(x)
    check(_fns()["bwd_tiles"](_dt(x), ptr(dv), ptr(v), ptr(_nhwc_view(dres) if dres is not None else None), M, C,
                              ptr(w32), ptr(stats), 1, ptr(part[0]), ptr(part[1]), T, ptr(kbuf), ptr(dx), ptr(dgb[0]),
                              ptr(dgb[1]), ptr(_nhwc_view(act) if act is not None else None),
                              stream_handle(x.device)), "mifx_bn_relu_bwd_tiles")
    return dx, dgb


def _bwd_any(ctx, dy, x, w32, stats, relu, dres):
    part = _take_tiles(ctx, dy) if relu else None
    dst = _grad_dests(ctx)
    if part is not None and x.dtype == torch.bfloat16 and _nhwc_view(dy) is not None:
        return _bwd_tiles(dy, x, w32, stats, dres, part, dst=dst)
    return _bwd(dy, x, w32, stats, relu, dres, dst=dst)


def _fwd_tiles(x, part, weight, bias, run_mean, run_var, momentum, eps, relu, apply=True):
    """Forward from per-tile statistics computed by the GEMM that produced x (mifx.ops.conv1x1): no statistics pass
    over x. part: [2, T, C] fp32 (tile means, tile M2), T tiles of M / T rows. apply=False: statistics (and running
    statistics) only, y None -- the consumer GEMM applies them to its operand (mifx.ops.conv1x1.bn_conv1x1)."""
    v = _nhwc_view(x)
    M, C = v.shape
    T = part.shape[1]
    w32, b32 = weight.float().contiguous(), bias.float().contiguous()
    stats = torch.empty(4, C, device=x.device, dtype=torch.float32)
    ws = torch.empty(_fns()["tiles_ws"](T, C), device=x.device, dtype=torch.float64)
    y = torch.empty_like(x) if apply else None
    check(_fns()["fwd_tiles"](_dt(x), ptr(v), M, C, ptr(part), T, M // T, ptr(w32), ptr(b32), float(eps),
                              float(momentum), ptr(run_mean), ptr(run_var if run_mean is not None else None),
                              int(relu), ptr(stats), ptr(ws), ptr(y), stream_handle(x.device)), "mifx_bn_relu_fwd_tiles")
    return y, w32, stats


class _BNReLUTiles(torch.autograd.Function):
    """(relu(bn(x)), x) with the batch statistics taken from the producing GEMM's per-tile partials. The second output
    aliases x: its consumer (the next block's identity shortcut, i.e. the residual operand of the next fused conv)
    sends its gradient back through here, and the BN backward kernel adds it in (its `dres` input), as _AddBNReLU
    does -- no separate gradient-sum kernel."""

    @staticmethod
    def forward(ctx, x, part, weight, bias, run_mean, run_var, momentum, eps):
        y, w32, stats = _fwd_tiles(x, part, weight, bias, run_mean, run_var, momentum, eps, True)
        ctx.save_for_backward(x, w32, stats)
        ctx.wdtype, ctx.mifx_bn, ctx.mifx_wb = weight.dtype, True, (weight, bias)
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(part)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        x, w32, stats = ctx.saved_tensors
        if dy is None:
            return dpass, None, None, None, None, None, None, None
        dx, dgb = _bwd_any(ctx, dy, x, w32, stats, True, dpass)
        return dx, None, dgb[0].to(ctx.wdtype), dgb[1].to(ctx.wdtype), None, None, None, None


class _BNReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, run_mean, run_var, momentum, eps, relu):
        y, _, w32, stats = _fwd(x, None, weight, bias, run_mean, run_var, momentum, eps, relu)
        ctx.save_for_backward(x, w32, stats)
        ctx.relu, ctx.wdtype, ctx.mifx_bn, ctx.mifx_wb = relu, weight.dtype, bool(relu), (weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32, stats = ctx.saved_tensors
        dx, dgb = _bwd_any(ctx, dy, x, w32, stats, ctx.relu, None)
        return dx, dgb[0].to(ctx.wdtype), dgb[1].to(ctx.wdtype), None, None, None, None, None


class _AddBNReLU(torch.autograd.Function):
    """(y, s) = (relu(bn(a + b)), a + b): the residual sum of a pre-activation block feeds both the next
    BN+ReLU and (often) the next identity shortcut. Forward: the add is done inside the statistics
    pass; backward: the shortcut's gradient ds is accumulated by the dx kernel, so neither direction
    launches a separate add kernel."""

    @staticmethod
    def forward(ctx, a, b, weight, bias, run_mean, run_var, momentum, eps):
        y, s, w32, stats = _fwd(a, b.to(a.dtype), weight, bias, run_mean, run_var, momentum, eps, True)
        ctx.save_for_backward(s, w32, stats)
        ctx.wdtype, ctx.mifx_bn, ctx.mifx_wb = weight.dtype, True, (weight, bias)
        # an unused output (s, when the next block has a projection shortcut) arrives as None instead of
        # a materialised zero tensor: autograd created those in NCHW, forcing a full channels_last copy
        # (plus a read of zeros) in the backward of the first block of every stage
        ctx.set_materialize_grads(False)
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, w32, stats = ctx.saved_tensors
        if dy is None:
            if ds is None:
                return None, None, None, None, None, None, None, None
            return ds, ds, None, None, None, None, None, None
        dx, dgb = _bwd_any(ctx, dy, s, w32, stats, True, ds)
        return dx, dx, dgb[0].to(ctx.wdtype), dgb[1].to(ctx.wdtype), None, None, None, None


def bn_relu(x, weight, bias, running_mean=None, running_var=None, training=True, momentum=0.1, eps=1e-5,
            relu=True):
    """relu(batch_norm(x)) (relu optional). Native on channels_last GPU tensors."""
    if native_ok(x):
        if training:
            return _BNReLU.apply(x, weight, bias, running_mean, running_var, momentum, eps, relu)
        scale = (weight.float() * torch.rsqrt(running_var.float() + eps)).contiguous()
        shift = (bias.float() - running_mean.float() * scale).contiguous()
        v = _nhwc_view(x)
        y = torch.empty_like(x)
        check(_fns()["apply"](_dt(x), ptr(v), v.shape[0], v.shape[1], ptr(scale), ptr(shift), int(relu), ptr(y),
                              stream_handle(x.device)), "mifx_bn_relu_apply")
        return y
    if x.is_cuda and _lib.gpu_available() and x.dim() == 4 and x.shape[1] % 8 == 0 \
            and x.is_contiguous(memory_format=torch.channels_last):
        _fns()  # channels_last GPU input that should have been native: fail loudly if the library is absent
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    return F.relu(y) if relu else y


def add_bn_relu(a, b, weight, bias, running_mean=None, running_var=None, training=True, momentum=0.1, eps=1e-5):
    """(relu(batch_norm(a + b)), a + b) with the add fused into the BN kernels on the GPU."""
    if training and native_ok(a) and b.shape == a.shape and native_ok(b.to(a.dtype)):
        return _AddBNReLU.apply(a, b, weight, bias, running_mean, running_var, momentum, eps)
    s = a + b
    return bn_relu(s, weight, bias, running_mean, running_var, training, momentum, eps, True), s


class BatchNormReLU2d(nn.BatchNorm2d):
    """nn.BatchNorm2d followed by ReLU, fused on the GPU. Parameters/buffers/state_dict == BatchNorm2d.
    `forward_add(a, b)` normalises the residual sum a + b and also returns it."""

    defer_count = False  # num_batches_tracked advanced by the caller (defer_batch_counts)

    def _args(self):
        if self.training and self.track_running_stats and not self.defer_count:
            self.num_batches_tracked.add_(1)
        use_batch_stats = self.training or not self.track_running_stats
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        return rm, rv, use_batch_stats

    def forward(self, x):
        rm, rv, train = self._args()
        return bn_relu(x, self.weight, self.bias, rm, rv, train, self.momentum, self.eps, True)

    def forward_add(self, a, b):
        rm, rv, train = self._args()
        return add_bn_relu(a, b, self.weight, self.bias, rm, rv, train, self.momentum, self.eps)

    def forward_tiles(self, x, part):
        """(relu(bn(x)), x) in training mode with x's batch statistics already reduced per tile by the GEMM that
        wrote it (part: [2, T, C], mifx.ops.conv1x1); other modes fall back to forward()."""
        rm, rv, train = self._args()
        if train and self.training and native_ok(x):
            return _BNReLUTiles.apply(x, part, self.weight, self.bias, rm, rv, self.momentum, self.eps)
        return bn_relu(x, self.weight, self.bias, rm, rv, train, self.momentum, self.eps, True), x


def defer_batch_counts(model: nn.Module) -> torch.Tensor | None:
    """Re-home every BatchNormReLU2d's `num_batches_tracked` as one element of a single int64 tensor and stop the
    per-forward increments: the caller advances them all with one `add_(1)` per training forward -- one kernel instead
    of one per BatchNorm (49 in ResNet-50: ~0.2 ms of a B=256 step, profiles/archive/resnet_steady_r4b.md). Call after the
    model reached its device. Returns the tensor (None without such BatchNorms)."""
    bns = [m for m in model.modules() if isinstance(m, BatchNormReLU2d) and m.track_running_stats]
    if not bns:
        return None
    flat = torch.stack([m.num_batches_tracked.detach().clone() for m in bns])
    for i, m in enumerate(bns):
        m._buffers["num_batches_tracked"] = flat[i]
        m.defer_count = True
    return flat
