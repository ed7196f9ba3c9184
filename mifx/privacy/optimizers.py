"""DP-SGD optimizers: per-microbatch gradients in ONE vectorised pass + fused clip/sum/noise.

Reference: `optimizers/dp_optimizer.py:24-100` — `make_optimizer_class(cls)` wraps an optimizer so
that `compute_gradients(vector_loss)` reshapes the loss to [num_microbatches, -1], computes each
microbatch's gradient in a sequential `tf.while_loop`, and feeds them through a
`GaussianAverageQuery(l2_norm_clip, l2_norm_clip * noise_multiplier, num_microbatches)`.

MI355X-first: the microbatch loop becomes `torch.func.vmap(grad(...))` — one batched backward
whose GEMMs have the microbatch as an extra batch dimension (MFMA-friendly), producing G[M, P];
the clip -> sum -> Gaussian noise -> /M chain is one HIP kernel pair over G (csrc/dp.hip) with an
in-kernel Philox stream (seed, step) so runs are reproducible. When G would exceed
`max_g_bytes` the microbatches are processed in chunks (noise added once at the end)."""
from __future__ import annotations

import math

import torch
from torch.func import functional_call, grad_and_value, vmap

from ..ops import dpsgd_mnist
from ..ops.dp import clip_sum_noise
from ..trainer.optim import make_optimizer
from .queries import GaussianAverageQuery

_MAX_FUSED_ROWS = 4096  # clip_sum_noise's row bound


def sparse_softmax_ce(logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
    """Per-example `tf.nn.sparse_softmax_cross_entropy_with_logits` (the tutorial's vector loss). Passing
    this function as `vector_loss_fn` lets models with a fused per-microbatch gradient kernel use it."""
    return torch.nn.functional.cross_entropy(logits, labels, reduction="none")


sparse_softmax_ce.mifx_kind = "sparse_softmax_ce"


class DPOptimizer:
    """Differentially-private wrapper around a torch optimizer.

    Usage::

        opt = DPOptimizer(torch.optim.SGD(model.parameters(), lr=0.1), l2_norm_clip=1.0,
                          noise_multiplier=1.1, num_microbatches=256)
        loss = opt.step(model, vector_loss_fn, x, y)   # vector_loss_fn(logits, y) -> [B]; 0-dim loss tensor
    """

    def __init__(self, optimizer: torch.optim.Optimizer, l2_norm_clip: float, noise_multiplier: float,
                 num_microbatches: int | None = None, seed: int | None = None, max_g_bytes: int = 8 << 30):
        self.optimizer = optimizer
        self.l2_norm_clip = float(l2_norm_clip)
        self.noise_multiplier = float(noise_multiplier)
        self.num_microbatches = num_microbatches
        self.seed = int(seed if seed is not None else torch.randint(0, 2 ** 62, (1,)).item())
        self.max_g_bytes = max_g_bytes
        self.steps = 0
        self.last_norms = None

    @property
    def param_groups(self):
        return self.optimizer.param_groups

    def zero_grad(self, set_to_none: bool = True) -> None:
        self.optimizer.zero_grad(set_to_none=set_to_none)

    def query(self, m: int) -> GaussianAverageQuery:
        """The equivalent (record-at-a-time) query this optimizer implements in one fused pass."""
        return GaussianAverageQuery(self.l2_norm_clip, self.l2_norm_clip * self.noise_multiplier, m)

    def compute_gradients(self, model: torch.nn.Module, vector_loss_fn, *batch) -> torch.Tensor:
        """Fill `p.grad` with the noised, clipped microbatch average; returns the mean example loss as a 0-dim
        tensor (read it with float(); no host synchronisation per step)."""
        B = batch[0].shape[0]
        M = self.num_microbatches or B
        if B % M:
            raise ValueError("Number of microbatches should divide evenly batch_size")
        if (getattr(vector_loss_fn, "mifx_kind", None) == "sparse_softmax_ce" and len(batch) == 2
                and M <= _MAX_FUSED_ROWS and dpsgd_mnist.supported(model, batch[0])):
            return self._fused_mnist(model, *batch, M)
        names = [n for n, p in model.named_parameters() if p.requires_grad]
        params = {n: p.detach() for n, p in model.named_parameters() if p.requires_grad}
        buffers = {n: b.detach() for n, b in model.named_buffers()}

        def mb_loss(p, *mb):
            out = functional_call(model, (p, buffers), (mb[0],))
            return vector_loss_fn(out, *mb[1:]).sum()

        per_mb = vmap(grad_and_value(mb_loss), in_dims=(None,) + (0,) * len(batch))
        split = [t.reshape(M, B // M, *t.shape[1:]) for t in batch]
        numel = sum(params[n].numel() for n in names)
        rows = max(1, min(M, self.max_g_bytes // max(1, numel * 4)))
        acc, total_loss, norms = None, None, []
        for r0 in range(0, M, rows):
            grads, losses = per_mb(params, *[t[r0:r0 + rows] for t in split])
            G = torch.cat([grads[n].reshape(grads[n].shape[0], -1).float() for n in names], dim=1)
            lsum = losses.detach().sum()
            total_loss = lsum if total_loss is None else total_loss + lsum
            if rows == M:  # whole batch in one fused pass: clip + sum + noise + /M
                acc, nrm = clip_sum_noise(G, self.l2_norm_clip, self.l2_norm_clip * self.noise_multiplier, M,
                                          self.seed, self.steps, return_norms=True)
                norms.append(nrm)
            else:
                part, nrm = clip_sum_noise(G, self.l2_norm_clip, 0.0, 1.0, return_norms=True)
                acc = part if acc is None else acc + part
                norms.append(nrm)
        if rows < M:  # noise once over the accumulated clipped sum, then normalise
            acc = clip_sum_noise(acc[None, :], math.inf, self.l2_norm_clip * self.noise_multiplier, M, self.seed,
                                 self.steps)
        self.last_norms = torch.cat(norms)
        self._assign_grads(model, names, acc)
        return total_loss / B

    @staticmethod
    def _assign_grads(model, names, acc) -> None:
        off = 0
        named = dict(model.named_parameters())
        for n in names:
            p = named[n]
            k = p.numel()
            g = acc[off:off + k].view_as(p).to(p.dtype)
            p.grad = g.clone() if p.grad is None else p.grad.copy_(g)
            off += k

    def _fused_mnist(self, model, x, y, M) -> torch.Tensor:
        """MNIST tutorial CNN on the GPU: all M microbatch gradients from one kernel (csrc/dpsgd_mnist.hip),
        then the same fused clip / sum / noise pass as the generic path, written straight into one flat gradient
        buffer whose slices become the parameters' .grad (no per-parameter copies, no host sync)."""
        G, losses = dpsgd_mnist.per_microbatch_grads(model, x, y, M, max_bytes=self.max_g_bytes)
        flat = getattr(self, "_flat_grad", None)
        if flat is None or flat.device != G.device:
            flat = self._flat_grad = torch.empty(G.shape[1], dtype=torch.float32, device=G.device)
        _, self.last_norms = clip_sum_noise(G, self.l2_norm_clip, self.l2_norm_clip * self.noise_multiplier, M,
                                            self.seed, self.steps, return_norms=True, out=flat)
        off = 0
        for p in model.parameters():
            p.grad = flat[off:off + p.numel()].view_as(p)
            off += p.numel()
        return losses.sum() / x.shape[0]

    def step(self, model: torch.nn.Module, vector_loss_fn, *batch) -> torch.Tensor:
        self.optimizer.zero_grad(set_to_none=True)
        loss = self.compute_gradients(model, vector_loss_fn, *batch)
        self.optimizer.step()
        self.steps += 1
        return loss


def make_optimizer_class(kind):
    """DP counterpart of an optimizer — the reference's `make_optimizer_class(tf.train.XOptimizer)`
    (`dp_optimizer.py:25-94`): `kind` is an optimizer name ('sgd', 'adagrad', 'adam', 'ftrl') or any
    `torch.optim.Optimizer` subclass (constructed as `cls(params, lr=learning_rate, **kw)`)."""
    if isinstance(kind, type) and issubclass(kind, torch.optim.Optimizer):
        def build(params, lr, **kw):
            return kind(params, lr=lr, **kw)

        label = kind.__name__
    elif isinstance(kind, str):
        def build(params, lr, **kw):
            return make_optimizer(kind, params, lr, **kw)

        label = kind.capitalize()
    else:
        raise TypeError(f"make_optimizer_class expects an optimizer name or torch.optim.Optimizer subclass, got "
                        f"{kind!r}")

    class _DP(DPOptimizer):
        def __init__(self, l2_norm_clip, noise_multiplier, num_microbatches, params, learning_rate, seed=None,
                     **kw):
            super().__init__(build(params, learning_rate, **kw), l2_norm_clip, noise_multiplier, num_microbatches,
                             seed)

    _DP.__name__ = _DP.__qualname__ = f"DP{label}Optimizer"
    return _DP


DPGradientDescentOptimizer = make_optimizer_class("sgd")
DPAdagradOptimizer = make_optimizer_class("adagrad")
DPAdamOptimizer = make_optimizer_class("adam")
