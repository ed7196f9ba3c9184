"""Per-microbatch gradients of the DP-SGD MNIST tutorial CNN in one HIP kernel (csrc/dpsgd_mnist.hip).

`per_microbatch_grads(model, x, y, M)` returns G [M, ld] (fp32, columns = the model's flattened
parameters in `named_parameters()` order, ld = NP rounded up to 4 with zero pad columns) and the
per-example softmax cross-entropy losses [B] — the same numbers as
``vmap(grad(sum of microbatch losses))`` over `mifx.models.cnn.MnistDPCNN`, computed with one
workgroup per microbatch instead of a batched autograd graph (reference
`dp_optimizer.py:59-90` runs one backward per microbatch in a while-loop).

GPU only: `supported()` says whether a model / batch can take this path."""
from __future__ import annotations

import functools

import torch

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle

NUM_PARAMS = 26010
LD = (NUM_PARAMS + 3) // 4 * 4
_SHAPES = [("conv1.weight", (16, 1, 8, 8)), ("conv1.bias", (16,)), ("conv2.weight", (32, 16, 4, 4)),
           ("conv2.bias", (32,)), ("fc1.weight", (32, 512)), ("fc1.bias", (32,)), ("fc2.weight", (10, 32)),
           ("fc2.bias", (10,))]


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("dpsgd_mnist")
    f = {
        "np": sig(lib, "mifx_dpmnist_num_params", []),
        "grads": sig(lib, "mifx_dpmnist_grads", [VP, VP, I32, I32] + [VP] * 8 + [VP, I32, VP, VP]),
    }
    assert f["np"]() == NUM_PARAMS, "dpsgd_mnist.hip parameter layout mismatch"
    return f


def supported(model: torch.nn.Module, x: torch.Tensor) -> bool:
    params = list(model.named_parameters())
    if [(n, tuple(p.shape)) for n, p in params] != _SHAPES:
        return False
    if not all(p.is_cuda and p.dtype == torch.float32 and p.requires_grad for _, p in params):
        return False
    return x.is_cuda and x.dtype == torch.float32 and x.shape[-2:] == (28, 28) and x.numel() == x.shape[0] * 784


def per_microbatch_grads(model: torch.nn.Module, x: torch.Tensor, y: torch.Tensor, num_microbatches: int,
                         max_bytes: int | None = None):
    """max_bytes bounds the per-example scratch [B, LD] fp32: above it the kernel writes the M microbatch rows
    directly (one workgroup per microbatch) instead of one row per example."""
    B = x.shape[0]
    M = int(num_microbatches)
    if B % M:
        raise ValueError("Number of microbatches should divide evenly batch_size")
    if not supported(model, x):
        raise ValueError("per_microbatch_grads needs an fp32 MnistDPCNN on the GPU and [B, (1,) 28, 28] fp32 input")
    ps = [p.detach().contiguous() for _, p in model.named_parameters()]
    xc = x.detach().contiguous()
    yc = y.detach().to(torch.int64).contiguous()
    # One workgroup per example (B workgroups fill the chip even when M is small), then the microbatch sums.
    rows = B if M < B and B <= 65536 else M
    if max_bytes is not None and rows != M and rows * LD * 4 > max_bytes:
        rows = M
    G = torch.empty(rows, LD, dtype=torch.float32, device=x.device)
    loss = torch.empty(B, dtype=torch.float32, device=x.device)
    check(_fns()["grads"](ptr(xc), ptr(yc), B, rows, *[ptr(p) for p in ps], ptr(G), LD, ptr(loss),
                          stream_handle(x.device)), "mifx_dpmnist_grads")
    if rows != M:
        G = G.view(M, B // M, LD).sum(1)
    return G, loss


def assign_mean_grads(model: torch.nn.Module, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Non-private step of the same network (the tutorial's `--dpsgd=False`): p.grad = gradient of the mean
    softmax cross-entropy, from the per-example kernel (one workgroup per example) and one column sum; returns
    the mean loss as a 0-dim tensor. GPU only (see `supported`)."""
    G, loss = per_microbatch_grads(model, x, y, 1)
    g = G[0] / x.shape[0]
    off = 0
    for p in model.parameters():
        p.grad = g[off:off + p.numel()].view_as(p)
        off += p.numel()
    return loss.mean()
