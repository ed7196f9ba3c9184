"""Megatron-style tensor parallelism over RCCL (one process per GPU, xGMI all-reduce).

No reference counterpart (TP absent in the reference); BASELINE config 4 asks for a
BERT-base fine-tune at TP=8, so this module provides the standard column/row split:

* `ColumnParallelLinear`: W split along the output dim; input replicated (identity forward,
  all-reduce of the input gradient backward); output stays sharded (or is all-gathered).
* `RowParallelLinear`: W split along the input dim; input sharded; partial outputs all-reduced
  forward (identity backward); bias added once after the reduction.
* `VocabParallelEmbedding`: vocabulary rows split; out-of-shard ids masked; all-reduce forward.
* `head_partition(n_heads, world)`: BERT-base has 12 heads, not divisible by 8 — heads are
  partitioned as evenly as possible (2,2,2,2,1,1,1,1 at TP=8) and the QKV / output projections
  use the matching uneven column / row splits, so TP=8 is exact (not approximate). Cost of the imbalance: the
  fused attention kernels take 13.2 + 22.1 us per layer for all 12 heads at B = 32, S = 128
  (profiles/archive/bert_steady_kernels_r3_fold.md), so a 2-head rank spends ~5.9 us per layer where an even 1.5-head
  share would take ~4.4: ~1.5 us per layer, ~18 us per 12-layer step, while the GEMMs and LayerNorms split evenly
  (the FFN's 3072 columns and the 768-wide activations divide by 8). Rebalancing would need heads split across
  ranks (extra all-to-alls per layer), which costs more than it saves at this size.

Sequence parallelism (BertConfig.sequence_parallel): the residual stream between the TP regions is split over the
ranks by token (gather_seq / reduce_scatter_seq / scatter_to_seq / gather_seq_replicated below; all_reduce_grads
sums the gradients of the parameters that act on token shards).

Two all-reduces per transformer block (after attention-out and FFN-out), each of
[tokens, hidden] activations — on MI355X the 8-GPU xGMI ring is ~7 links x ~150 GB/s, so a
[32*128, 768] bf16 block reduction (6.3 MB) is ~10-15 us. On the peer-memory path those two run OVERLAPPED with their
row-parallel GEMMs: `gemm_allreduce_overlapped` computes the GEMM in token chunks and reduces chunk i on a side stream
while chunk i+1 computes (mifx.ops.gemm.linear / ffn with tp=...; tools/tp_kernel_table.py reports how much of the
all-reduce kernels' time runs concurrently with GEMMs).

`TPGroup.enable_ipc(max_elems, device)` moves every bf16 TP all-reduce onto the two-shot peer-memory kernels of
mifx.parallel.tp_ipc (no host collective: the TP step captures into a hipGraph); otherwise torch.distributed's
all-reduce runs in place on the fresh GEMM output / gradient (no defensive copies either way)."""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ..ops import fused_bert as fb


class TPGroup:
    """The tensor-parallel process group (default: WORLD, or a single-rank no-op group)."""

    def __init__(self, group=None):
        self.group = group if group is not None else (dist.group.WORLD if dist.is_initialized() else None)
        self.size = dist.get_world_size(self.group) if self.group is not None else 1
        self.rank = dist.get_rank(self.group) if self.group is not None else 0
        self.ipc = None

    def enable_ipc(self, max_elems: int, device) -> None:
        """Route bf16 all-reduces of up to max_elems elements through the peer-memory kernels (collective)."""
        if self.size > 1 and self.ipc is None:
            from .tp_ipc import IpcAllReduce

            self.ipc = IpcAllReduce(self.group, device, max_elems)

    def disable_ipc(self) -> None:
        if self.ipc is not None:
            self.ipc.close()
            self.ipc = None

    def check(self) -> None:
        if self.ipc is not None:
            self.ipc.check()


def ipc_eligible(x: torch.Tensor, tp: TPGroup) -> bool:
    """The all-reduce of x runs on the peer-memory kernels (which write a NEW tensor); otherwise torch.distributed
    reduces x IN PLACE."""
    return (tp.ipc is not None and x.dtype == torch.bfloat16 and x.is_cuda and x.numel() % 4 == 0
            and x.numel() <= tp.ipc.npad)


def _all_reduce(x: torch.Tensor, tp: TPGroup) -> torch.Tensor:
    """Sum over the TP ranks. x must be a fresh tensor nobody else reads (a GEMM output or an incoming gradient):
    the torch path reduces it in place, the IPC path returns a new tensor."""
    if tp.size == 1:
        return x
    x = x.contiguous()
    if ipc_eligible(x, tp):
        return tp.ipc.all_reduce(x)
    dist.all_reduce(x, group=tp.group)
    return x


# Row-parallel GEMM + all-reduce overlap (TP > 1 on the peer-memory kernels): the GEMM runs in token chunks on the
# compute stream and each chunk's all-reduce on a side stream as soon as the chunk is written, so chunk i's exchange
# overlaps chunk i+1's GEMM; the compute stream joins the side stream before the reduced activation is used (no other
# all-reduce of the group can then be in flight: the kernels' epochs stay in issue order). Graph-capturable (event
# fork / join). MIFX_TP_OVERLAP_CHUNKS: chunks per GEMM -- opt-in (default 1 = the plain GEMM-then-all-reduce). For
# BERT-base at TP = 8 the row-parallel GEMM chunks are ~1 us (4096 x 768 x 96 split in 4), too short to hide an
# all-reduce behind, while chunking multiplies the all-reduce launches by 4; on the one-GPU rehearsal (ranks sharing
# the device) the chunked step measured slower (TP=2: 38.1 vs 13.2 ms eager, profiles/bert_tp2_overlap_r5.md /
# bert_tp2_nooverlap_r5.md). It pays where a chunk's GEMM outlasts its all-reduce (wider models, separate GPUs).
_OVERLAP_CHUNKS = int(os.environ.get("MIFX_TP_OVERLAP_CHUNKS", "1"))
_SIDE: dict = {}


def overlap_ok(tp: TPGroup | None, M: int, N: int) -> bool:
    """The row-parallel product [M, N] can be reduced chunk-by-chunk on the peer-memory kernels."""
    return (tp is not None and tp.size > 1 and tp.ipc is not None and _OVERLAP_CHUNKS > 1 and M % (64 * _OVERLAP_CHUNKS) == 0
            and (M // _OVERLAP_CHUNKS) * N <= tp.ipc.npad and N % 4 == 0)


def gemm_allreduce_overlapped(x2: torch.Tensor, gemm, N: int, tp: TPGroup) -> torch.Tensor:
    """all_reduce(gemm(x2)) over the TP group, gemm: [m, K] -> [m, N] bf16 on the current stream, applied to token
    chunks whose all-reduces run on a side stream (see above). Returns the reduced [M, N] (a new tensor)."""
    M = x2.shape[0]
    dev = x2.device
    main = torch.cuda.current_stream(dev)
    side = _SIDE.get(dev)
    if side is None:
        side = _SIDE[dev] = torch.cuda.Stream(dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    r0 = 0
    for r in split_sizes(M, _OVERLAP_CHUNKS, 64):
        part = gemm(x2[r0:r0 + r])
        ev = torch.cuda.Event()
        ev.record(main)
        side.wait_event(ev)
        with torch.cuda.stream(side):
            tp.ipc.all_reduce(part, out=y[r0:r0 + r])
        part.record_stream(side)
        r0 += r
    main.wait_stream(side)
    return y


class _CopyToTP(torch.autograd.Function):
    """identity forward, all-reduce backward (Megatron's `f`)."""

    @staticmethod
    def forward(ctx, x, tp):
        ctx.tp = tp
        return x

    @staticmethod
    def backward(ctx, g):
        # (the incoming gradient may be shared by other consumers of the graph: reduce a private copy whenever the
        # in-place torch path will run -- no IPC group, or a tensor the IPC kernels do not take; the IPC path writes
        # a new tensor anyway)
        if ctx.tp.size > 1 and not ipc_eligible(g.contiguous(), ctx.tp):
            g = g.clone()
        return _all_reduce(g, ctx.tp), None


class _ReduceFromTP(torch.autograd.Function):
    """all-reduce forward, identity backward (Megatron's `g`)."""

    @staticmethod
    def forward(ctx, x, tp):
        # x is the row-parallel GEMM's fresh output (F.linear saves its input and weight, not its output): the
        # torch path reduces it in place (marked dirty for autograd), the IPC path writes a new tensor
        y = _all_reduce(x, tp)
        if y is x:
            ctx.mark_dirty(x)
        return y

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherFromTP(torch.autograd.Function):
    """all-gather along the last dim forward (uneven sizes allowed), slice backward."""

    @staticmethod
    def forward(ctx, x, tp, sizes):
        ctx.tp, ctx.sizes = tp, sizes
        if tp.size == 1:
            return x
        mx = max(sizes)
        pad = F.pad(x, (0, mx - x.shape[-1])).contiguous()
        outs = [torch.empty_like(pad) for _ in range(tp.size)]
        dist.all_gather(outs, pad, group=tp.group)
        return torch.cat([o[..., :s] for o, s in zip(outs, sizes)], -1)

    @staticmethod
    def backward(ctx, g):
        if ctx.tp.size == 1:
            return g, None, None
        off = sum(ctx.sizes[:ctx.tp.rank])
        return g[..., off:off + ctx.sizes[ctx.tp.rank]].contiguous(), None, None


# ---------------------------------------------------------------------------------------------- sequence parallelism
# Megatron-style sequence parallelism (Korthikanti et al. 2022): between the tensor-parallel regions the residual
# stream is split along the token dim -- rank r holds tokens [r T / W, (r + 1) T / W) of the token-major [T, H]
# activation -- so the LayerNorms, dropouts and residual adds run on 1/W of the tokens and their activations are
# stored once per rank instead of W times. Each row-parallel all-reduce becomes a reduce-scatter into the token shard
# and each column-parallel input an all-gather of it (same bytes on the wire as the all-reduce it replaces: a ring
# all-reduce IS reduce-scatter + all-gather). On the peer-memory path these are csrc/tp_allreduce.hip's
# reduce-scatter / all-gather kernels (graph-capturable); otherwise torch.distributed.


def _seq_rows(T: int, tp: TPGroup) -> int:
    if T % tp.size:
        raise ValueError(f"sequence parallelism: {T} tokens do not split over {tp.size} ranks")
    return T // tp.size


def _ipc_shard_ok(x: torch.Tensor, n: int, tp: TPGroup) -> bool:
    return tp.ipc is not None and x.dtype == torch.bfloat16 and x.is_cuda and tp.ipc.shard_ok(n)


def seq_reduce_scatter(x: torch.Tensor, tp: TPGroup) -> torch.Tensor:
    """[T, ...] partial sums on every rank -> this rank's [T / W, ...] token rows of their sum."""
    x = x.contiguous()
    Ts = _seq_rows(x.shape[0], tp)
    if _ipc_shard_ok(x, x.numel(), tp):
        return tp.ipc.reduce_scatter(x).view(Ts, *x.shape[1:])
    if dist.get_backend(tp.group) == "nccl":
        y = x.new_empty(Ts, *x.shape[1:])
        dist.reduce_scatter_tensor(y, x, group=tp.group)
        return y
    y = x.clone()  # gloo has no reduce-scatter: all-reduce a private copy, keep the own rows
    dist.all_reduce(y, group=tp.group)
    return y[tp.rank * Ts:(tp.rank + 1) * Ts].contiguous()


def seq_all_gather(x: torch.Tensor, tp: TPGroup) -> torch.Tensor:
    """This rank's [T / W, ...] token rows -> the full [T, ...] (rank-order concatenation)."""
    x = x.contiguous()
    T = x.shape[0] * tp.size
    if _ipc_shard_ok(x, x.numel() * tp.size, tp):
        return tp.ipc.all_gather(x).view(T, *x.shape[1:])
    y = x.new_empty(T, *x.shape[1:])
    if dist.get_backend(tp.group) == "nccl":
        dist.all_gather_into_tensor(y, x, group=tp.group)
    else:
        dist.all_gather(list(y.chunk(tp.size)), x, group=tp.group)
    return y


class _GatherSeq(torch.autograd.Function):
    """all-gather of the token shards forward, reduce-scatter of the (partial, per-rank) gradient backward: the input of
    a column-parallel projection (replaces copy_to_tp)."""

    @staticmethod
    def forward(ctx, x, tp):
        ctx.tp = tp
        return seq_all_gather(x, tp)

    @staticmethod
    def backward(ctx, g):
        return seq_reduce_scatter(g, ctx.tp), None


class _ReduceScatterSeq(torch.autograd.Function):
    """reduce-scatter into the token shard forward, all-gather of the shard gradients backward: the output of a
    row-parallel projection (replaces reduce_from_tp)."""

    @staticmethod
    def forward(ctx, x, tp):
        ctx.tp = tp
        return seq_reduce_scatter(x, tp)

    @staticmethod
    def backward(ctx, g):
        return seq_all_gather(g, ctx.tp), None


class _ScatterToSeq(torch.autograd.Function):
    """replicated [T, ...] -> own token rows (cast to `dtype`) forward; all-gather backward (every rank's gradient of
    the replicated input is the concatenation of the shard gradients, so the replicated region's backward stays
    identical on every rank)."""

    @staticmethod
    def forward(ctx, x, tp, dtype):
        ctx.tp, ctx.dtype = tp, x.dtype
        Ts = _seq_rows(x.shape[0], tp)
        y = x[tp.rank * Ts:(tp.rank + 1) * Ts]
        # always a new tensor: an input already in `dtype` would otherwise come back as a VIEW of the replicated
        # activation (a custom Function's output aliasing its input)
        return y.to(dtype).contiguous() if y.dtype != dtype else y.clone(memory_format=torch.contiguous_format)

    @staticmethod
    def backward(ctx, g):
        return seq_all_gather(g, ctx.tp).to(ctx.dtype), None, None


class _GatherSeqReplicated(torch.autograd.Function):
    """token shards -> the replicated [T, ...] forward (into a replicated region: pooler / head); backward keeps the
    own rows of the (identical on every rank) gradient."""

    @staticmethod
    def forward(ctx, x, tp):
        ctx.tp = tp
        return seq_all_gather(x, tp)

    @staticmethod
    def backward(ctx, g):
        Ts = g.shape[0] // ctx.tp.size
        return g[ctx.tp.rank * Ts:(ctx.tp.rank + 1) * Ts].contiguous(), None


def gather_seq(x, tp: TPGroup):
    return _GatherSeq.apply(x, tp)


def reduce_scatter_seq(x, tp: TPGroup):
    return _ReduceScatterSeq.apply(x, tp)


def scatter_to_seq(x, tp: TPGroup, dtype=None):
    return _ScatterToSeq.apply(x, tp, x.dtype if dtype is None else dtype)


def gather_seq_replicated(x, tp: TPGroup):
    return _GatherSeqReplicated.apply(x, tp)


@torch.no_grad()
def all_reduce_grads(params, tp: TPGroup) -> None:
    """Sum the gradients of `params` over the TP group in place, one collective per dtype: the parameters that act on
    token shards under sequence parallelism (LayerNorm weights / biases, row-parallel biases) get partial gradients
    from their rank's tokens. Graph-capturable on the peer-memory path (the gradients keep their addresses)."""
    if tp.size == 1:
        return
    by_dtype: dict = {}
    for p in params:
        if p.grad is not None:
            by_dtype.setdefault(p.grad.dtype, []).append(p.grad)
    for gs in by_dtype.values():
        flat = torch.cat([g.reshape(-1) for g in gs])
        pad = (-flat.numel()) % 4  # the IPC kernels move 4 bf16 per lane
        if pad:
            flat = F.pad(flat, (0, pad))
        sizes = [g.numel() for g in gs]
        flat = _all_reduce(flat, tp)[:sum(sizes)]
        torch._foreach_copy_(gs, [v.view_as(g) for v, g in zip(flat.split(sizes), gs)])


def copy_to_tp(x, tp: TPGroup):
    return _CopyToTP.apply(x, tp) if tp.size > 1 else x


def reduce_from_tp(x, tp: TPGroup):
    return _ReduceFromTP.apply(x, tp) if tp.size > 1 else x


def gather_from_tp(x, tp: TPGroup, sizes):
    return _GatherFromTP.apply(x, tp, list(sizes)) if tp.size > 1 else x


def split_sizes(n: int, parts: int, unit: int = 1) -> list[int]:
    """Split n (a multiple of `unit`) into `parts` chunks of whole units, as even as possible."""
    units = n // unit
    base, extra = divmod(units, parts)
    return [(base + (1 if i < extra else 0)) * unit for i in range(parts)]


def head_partition(n_heads: int, world: int) -> list[int]:
    return split_sizes(n_heads, world)


class ColumnParallelLinear(nn.Module):
    """y_shard = x @ W[:, shard] (+ b[shard]); `sizes` gives each rank's output width."""

    def __init__(self, in_features: int, out_features: int, tp: TPGroup, bias: bool = True, sizes=None,
                 gather_output: bool = False):
        super().__init__()
        self.tp, self.in_features, self.out_features = tp, in_features, out_features
        self.sizes = list(sizes) if sizes is not None else split_sizes(out_features, tp.size)
        self.local = self.sizes[tp.rank]
        self.offset = sum(self.sizes[:tp.rank])
        self.gather_output = gather_output
        self.weight = nn.Parameter(torch.empty(self.local, in_features))
        self.bias = nn.Parameter(torch.zeros(self.local)) if bias else None

    def load_full(self, weight: torch.Tensor, bias: torch.Tensor | None) -> None:
        with torch.no_grad():
            self.weight.copy_(weight[self.offset:self.offset + self.local])
            if self.bias is not None and bias is not None:
                self.bias.copy_(bias[self.offset:self.offset + self.local])

    def forward(self, x):
        y = fb.linear(copy_to_tp(x, self.tp), self.weight, self.bias)
        return gather_from_tp(y, self.tp, self.sizes) if self.gather_output else y


class RowParallelLinear(nn.Module):
    """y = all_reduce(x_shard @ W[shard, :]^T) + b; `sizes` gives each rank's input width."""

    def __init__(self, in_features: int, out_features: int, tp: TPGroup, bias: bool = True, sizes=None):
        super().__init__()
        self.tp, self.in_features, self.out_features = tp, in_features, out_features
        self.sizes = list(sizes) if sizes is not None else split_sizes(in_features, tp.size)
        self.local = self.sizes[tp.rank]
        self.offset = sum(self.sizes[:tp.rank])
        self.weight = nn.Parameter(torch.empty(out_features, self.local))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None

    def load_full(self, weight: torch.Tensor, bias: torch.Tensor | None) -> None:
        with torch.no_grad():
            self.weight.copy_(weight[:, self.offset:self.offset + self.local])
            if self.bias is not None and bias is not None:
                self.bias.copy_(bias)

    def forward(self, x_shard, add_bias: bool = True):
        """add_bias=False returns the reduced partial products only (the caller fuses the bias, e.g. into
        fb.bias_dropout_add_layernorm)."""
        y = reduce_from_tp(F.linear(x_shard, self.weight), self.tp)
        # add the bias in the activation dtype (keeps a bf16 residual stream under autocast); its gradient
        # is a deterministic HIP column reduction on the GPU
        return fb.bias_add(y, self.bias) if (self.bias is not None and add_bias) else y


class VocabParallelEmbedding(nn.Module):
    def __init__(self, num_embeddings: int, dim: int, tp: TPGroup):
        super().__init__()
        self.tp, self.num_embeddings, self.dim = tp, num_embeddings, dim
        self.sizes = split_sizes(num_embeddings, tp.size)
        self.local = self.sizes[tp.rank]
        self.offset = sum(self.sizes[:tp.rank])
        self.weight = nn.Parameter(torch.empty(self.local, dim))

    def load_full(self, weight: torch.Tensor) -> None:
        with torch.no_grad():
            self.weight.copy_(weight[self.offset:self.offset + self.local])

    def forward(self, ids):
        if self.tp.size == 1:
            return fb.embedding(ids, self.weight)
        local = ids - self.offset
        mask = (local < 0) | (local >= self.local)
        out = fb.embedding(local.clamp(0, self.local - 1), self.weight)
        out = out.masked_fill(mask.unsqueeze(-1), 0.0)
        return reduce_from_tp(out, self.tp)
