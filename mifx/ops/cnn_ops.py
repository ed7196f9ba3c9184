"""Small-CNN training ops (csrc/cnn_ops.hip): fused softmax cross-entropy (loss + dlogits in one
pass), TF-semantics LRN forward/backward on NHWC activations, and a fused multi-tensor SGD + EMA
shadow-weight update (PATE `deep_cnn`, DP-SGD MNIST, Fashion-MNIST).

On a GPU the HIP kernels run (and a missing library raises); on CPU each op runs the PyTorch
reference of the same math, which the GPU tests compare against."""
from __future__ import annotations

import functools

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("cnn_ops")
    return {
        "xent": sig(lib, "mifx_cnn_softmax_xent", [I32, VP, VP, I32, I32, VP, VP, VP]),
        "lrn_fwd": sig(lib, "mifx_cnn_lrn_fwd", [I32, VP, I64, I32, I32, F32, F32, F32, VP, VP, VP]),
        "lrn_bwd": sig(lib, "mifx_cnn_lrn_bwd", [I32, VP, VP, VP, I64, I32, I32, F32, F32, VP, VP]),
        "chunk": sig(lib, "mifx_cnn_chunk_elems", []),
        "sgd_ema": sig(lib, "mifx_cnn_sgd_ema", [VP, VP, VP, I32, F32, F32, F32, VP]),
        "lrn_v8_ok": sig(lib, "mifx_cnn_lrn_v8_ok", [I32, I32]),
        "lrn_fwd_v8": sig(lib, "mifx_cnn_lrn_fwd_v8", [VP, I64, I32, F32, F32, F32, VP, VP]),
        "lrn_bwd_v8": sig(lib, "mifx_cnn_lrn_bwd_v8", [VP, VP, I64, I32, F32, F32, F32, VP, VP]),
        "tref": sig(lib, "mifx_cnn_tensor_ref_bytes", []),
    }


def _dt(t: torch.Tensor) -> int | None:
    return {torch.float32: 0, torch.bfloat16: 1}.get(t.dtype)


# ------------------------------------------------------------------ softmax cross-entropy
class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, reduction):
        x = logits.contiguous()
        lab = labels.contiguous().long()
        B, C = x.shape
        loss = torch.empty(B, device=x.device, dtype=torch.float32)
        d = torch.empty_like(x)
        check(_fns()["xent"](_dt(x), ptr(x), ptr(lab), B, C, ptr(loss), ptr(d), stream_handle(x.device)),
              "mifx_cnn_softmax_xent")
        ctx.reduction = reduction
        if reduction == "none":
            ctx.save_for_backward(d)
            return loss
        n = ((lab >= 0) & (lab < C)).sum().clamp_min(1).to(torch.float32) if reduction == "mean" else None
        ctx.save_for_backward(d, n) if n is not None else ctx.save_for_backward(d)
        return loss.sum() / n if n is not None else loss.sum()

    @staticmethod
    def backward(ctx, g):
        if ctx.reduction == "none":
            (d,) = ctx.saved_tensors
            return d * g.unsqueeze(1).to(d.dtype), None, None
        if ctx.reduction == "mean":
            d, n = ctx.saved_tensors
            return d * (g / n).to(d.dtype), None, None
        (d,) = ctx.saved_tensors
        return d * g.to(d.dtype), None, None


def softmax_cross_entropy(logits: torch.Tensor, labels: torch.Tensor, reduction: str = "mean") -> torch.Tensor:
    """== F.cross_entropy(logits, labels, reduction=...) (ignore_index -100 / out-of-range labels
    contribute nothing). GPU: one kernel computes the row losses and dlogits together."""
    if reduction not in ("mean", "sum", "none"):
        raise ValueError(reduction)
    if logits.is_cuda and logits.dim() == 2 and _dt(logits) is not None:
        return _SoftmaxXent.apply(logits, labels, reduction)
    return F.cross_entropy(logits.float(), labels.long(), reduction=reduction)


# ------------------------------------------------------------------------------------ LRN
def _nhwc(x: torch.Tensor) -> torch.Tensor | None:
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = x.shape
        return x.permute(0, 2, 3, 1).reshape(n * h * w, c)
    return None


class _LRN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, bias, alpha, beta):
        v = _nhwc(x)
        M, C = v.shape
        y = torch.empty_like(x)
        if x.dtype == torch.bfloat16 and x.data_ptr() % 16 == 0 and _fns()["lrn_v8_ok"](C, r):
            # vectorised bf16 kernels; backward recomputes the normaliser (nothing but x is saved)
            check(_fns()["lrn_fwd_v8"](ptr(v), M, C, bias, alpha, beta, ptr(_nhwc(y)), stream_handle(x.device)),
                  "mifx_cnn_lrn_fwd_v8")
            ctx.save_for_backward(x)
            ctx.args = (r, alpha, beta, bias, True)
            return y
        nrm = torch.empty(M, C, device=x.device, dtype=torch.float32)
        check(_fns()["lrn_fwd"](_dt(x), ptr(v), M, C, r, bias, alpha, beta, ptr(_nhwc(y)), ptr(nrm),
                                stream_handle(x.device)), "mifx_cnn_lrn_fwd")
        ctx.save_for_backward(x, nrm)
        ctx.args = (r, alpha, beta, bias, False)
        return y

    @staticmethod
    def backward(ctx, dy):
        r, alpha, beta, bias, v8 = ctx.args
        if v8:
            (x,) = ctx.saved_tensors
            dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
            dx = torch.empty_like(x)
            M, C = _nhwc(x).shape
            check(_fns()["lrn_bwd_v8"](ptr(_nhwc(x)), ptr(_nhwc(dy)), M, C, bias, alpha, beta, ptr(_nhwc(dx)),
                                       stream_handle(x.device)), "mifx_cnn_lrn_bwd_v8")
            return dx, None, None, None, None
        x, nrm = ctx.saved_tensors
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        M, C = nrm.shape
        dx = torch.empty_like(x)
        check(_fns()["lrn_bwd"](_dt(x), ptr(_nhwc(x)), ptr(_nhwc(dy)), ptr(nrm), M, C, r, alpha, beta,
                                ptr(_nhwc(dx)), stream_handle(x.device)), "mifx_cnn_lrn_bwd")
        return dx, None, None, None, None


def lrn(x: torch.Tensor, depth_radius: int = 5, bias: float = 1.0, alpha: float = 1.0, beta: float = 0.5):
    """tf.nn.lrn semantics over the channel dim of an NCHW-shaped tensor:
    y = x / (bias + alpha * sum_{|j-c|<=depth_radius} x_j^2) ** beta."""
    if x.is_cuda and _dt(x) is not None and _nhwc(x) is not None and x.data_ptr() % 4 == 0:
        return _LRN.apply(x, int(depth_radius), float(bias), float(alpha), float(beta))
    size = 2 * depth_radius + 1  # torch divides alpha by size
    return F.local_response_norm(x, size=size, alpha=alpha * size, beta=beta, k=bias)


# ------------------------------------------------------------------------- SGD + EMA
class SGDEMA:
    """Plain SGD (optional L2 weight decay) whose step also advances an EMA of every parameter:
    w -= lr * (g + wd * w); shadow += (1 - decay) * (w - shadow) — one multi-tensor HIP launch per step
    for fp32 GPU parameters (`deep_cnn.py:397-422`: GradientDescent + ExponentialMovingAverage)."""

    def __init__(self, params, lr: float, weight_decay: float = 0.0, ema: bool = True):
        self.params = [p for p in params if p.requires_grad]
        self.lr, self.weight_decay = float(lr), float(weight_decay)
        self.shadow = [p.detach().clone() for p in self.params] if ema else None
        self._key = None
        self._tabs = None
        self.native = bool(self.params) and all(p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()
                                                for p in self.params)

    def zero_grad(self, set_to_none: bool = True) -> None:
        """Default: drop the gradients, so backward writes fresh ones instead of a zero-fill + accumulate pass
        per parameter (for the 250-teacher ensemble's 600M-parameter dense layer that is ~1.7 ms a step). The
        launch table is keyed by the gradient addresses and rebuilt only when they change."""
        for p in self.params:
            if p.grad is not None:
                if set_to_none:
                    p.grad = None
                else:
                    p.grad.zero_()

    def _tables(self):
        for p in self.params:
            if not p.grad.is_contiguous():
                p.grad = p.grad.contiguous()
        key = tuple((p.data_ptr(), p.grad.data_ptr()) for p in self.params)
        if key == self._key:
            return self._tabs
        f = _fns()
        dev = self.params[0].device
        if self._tabs is None:  # chunk -> tensor index / start: fixed by the parameter sizes
            chunk = f["chunk"]()
            assert f["tref"]() == 32, "TensorRef layout mismatch"
            tix, cst = [], []
            for i, p in enumerate(self.params):
                for c0 in range(0, p.numel(), chunk):
                    tix.append(i)
                    cst.append(c0)
            self._chunks = (torch.tensor(tix, dtype=torch.int32).to(dev), torch.tensor(cst, dtype=torch.int64).to(dev))
        refs = []
        for i, p in enumerate(self.params):
            s = self.shadow[i].data_ptr() if self.shadow is not None else 0
            refs += [p.data_ptr(), p.grad.data_ptr(), s, p.numel()]
        # gradients are fresh tensors each step (zero_grad drops them), so their addresses can change: the table
        # goes up through pinned memory, stream-ordered, without stalling the host on the GPU
        tabs = torch.tensor(refs, dtype=torch.int64).pin_memory().to(dev, non_blocking=True)
        self._tabs = (tabs,) + self._chunks
        self._key = key
        return self._tabs

    @torch.no_grad()
    def step(self, lr: float | None = None, decay: float = 0.0) -> None:
        lr = self.lr if lr is None else float(lr)
        live = [p.grad is not None for p in self.params]
        if not all(live):
            for p in self.params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
        if self.native:
            tabs, tix, cst = self._tables()
            check(_fns()["sgd_ema"](ptr(tabs), ptr(tix), ptr(cst), int(tix.numel()), lr, 1.0 - float(decay),
                                    self.weight_decay, stream_handle(self.params[0].device)), "mifx_cnn_sgd_ema")
            return
        for i, p in enumerate(self.params):
            p.add_(p.grad + self.weight_decay * p, alpha=-lr)
            if self.shadow is not None:
                self.shadow[i].lerp_(p, 1.0 - float(decay))

