"""BERT (base by default) encoder + sequence-classification head, tensor-parallel over RCCL.

BASELINE config 4 ("BERT-base fine-tune Trainer component, TP=8"); there is no BERT in the
reference, so this follows the public BERT-base architecture: 12 layers, hidden 768, 12 heads,
FFN 3072, vocab 30522, 512 positions, 2 token types, post-LN, GELU(erf).

Per layer on each TP rank: one fused QKV column-parallel GEMM for the rank's heads (uneven head
split when heads % tp != 0), SDPA on the local heads, row-parallel output projection (+1
all-reduce), fused residual-add + LayerNorm (HIP), column-parallel FFN-in with fused bias+GELU
(HIP), row-parallel FFN-out (+1 all-reduce), fused residual-add + LayerNorm. With
`sequence_parallel=True` (TP > 1) each all-reduce is a reduce-scatter into the rank's token shard, the LayerNorms /
dropouts / residual adds run on that shard, and an all-gather feeds the next column-parallel projection
(BertLayer.forward_sp)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import fused_bert as fb
from ..ops import gemm as hg
from ..parallel.tensor_parallel import (ColumnParallelLinear, RowParallelLinear, TPGroup, VocabParallelEmbedding,
                                        all_reduce_grads, copy_to_tp, gather_seq, gather_seq_replicated,
                                        head_partition, overlap_ok, reduce_from_tp, reduce_scatter_seq, scatter_to_seq,
                                        split_sizes)


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    intermediate: int = 3072
    max_position: int = 512
    type_vocab: int = 2
    dropout: float = 0.1
    attn_dropout: float | None = None  # attention-probability dropout (None: same as dropout)
    dropout_seed: int = 1234  # dropout mask seed (identical on every TP rank)
    fused_attention: bool = True  # csrc/attention.hip (False: torch scaled_dot_product_attention)
    # forward projections on the hand-written MFMA GEMM (csrc/gemm.hip; FFN-in with bias + GELU fused into its
    # epilogue) for the shapes where it measured faster (mifx.ops.gemm.TUNED); None: on unless MIFX_BERT_HIP_GEMM=0
    hip_gemm: bool | None = None
    # residual gradients folded into the projections' input-gradient GEMMs (mifx.ops.gemm.GradSlot); off with
    # MIFX_BERT_FOLD_RESIDUAL=0
    fold_residual_grad: bool = field(
        default_factory=lambda: os.environ.get("MIFX_BERT_FOLD_RESIDUAL", "1") != "0")
    # sequence parallelism at TP > 1 (mifx.parallel.tensor_parallel): the residual stream, LayerNorms and hidden
    # dropouts run on each rank's 1/TP of the tokens; all-reduces become reduce-scatter + all-gather pairs
    sequence_parallel: bool = False
    num_labels: int = 2
    ln_eps: float = 1e-12
    init_std: float = 0.02

    @staticmethod
    def tiny(**kw) -> "BertConfig":
        d = dict(vocab_size=1000, hidden=64, layers=2, heads=4, intermediate=128, max_position=64)
        d.update(kw)
        return BertConfig(**d)


class BertLayer(nn.Module):
    def __init__(self, cfg: BertConfig, tp: TPGroup):
        super().__init__()
        self.cfg, self.tp = cfg, tp
        self.head_dim = cfg.hidden // cfg.heads
        self.heads_per_rank = head_partition(cfg.heads, tp.size)
        self.local_heads = self.heads_per_rank[tp.rank]
        hs = [h * self.head_dim for h in self.heads_per_rank]
        self.qkv = ColumnParallelLinear(cfg.hidden, 3 * cfg.hidden, tp, sizes=[3 * s for s in hs])
        self.attn_out = RowParallelLinear(cfg.hidden, cfg.hidden, tp, sizes=hs)
        self.ln1 = nn.LayerNorm(cfg.hidden, eps=cfg.ln_eps)
        self.ffn_in = ColumnParallelLinear(cfg.hidden, cfg.intermediate, tp,
                                           sizes=split_sizes(cfg.intermediate, tp.size))
        self.ffn_out = RowParallelLinear(cfg.intermediate, cfg.hidden, tp, sizes=self.ffn_in.sizes)
        self.ln2 = nn.LayerNorm(cfg.hidden, eps=cfg.ln_eps)

    def load_full(self, sd: dict, prefix: str) -> None:
        """Shard a full (TP=1) layer state dict into this rank's pieces."""
        H, d = self.cfg.hidden, self.head_dim
        w, b = sd[prefix + "qkv.weight"], sd[prefix + "qkv.bias"]
        h0 = sum(self.heads_per_rank[:self.tp.rank])
        rows = torch.cat([torch.arange(k * H + h0 * d, k * H + (h0 + self.local_heads) * d) for k in range(3)])
        with torch.no_grad():
            self.qkv.weight.copy_(w[rows])
            self.qkv.bias.copy_(b[rows])
        self.attn_out.load_full(sd[prefix + "attn_out.weight"], sd[prefix + "attn_out.bias"])
        self.ffn_in.load_full(sd[prefix + "ffn_in.weight"], sd[prefix + "ffn_in.bias"])
        self.ffn_out.load_full(sd[prefix + "ffn_out.weight"], sd[prefix + "ffn_out.bias"])
        for n in ("ln1", "ln2"):
            getattr(self, n).load_state_dict({"weight": sd[f"{prefix}{n}.weight"], "bias": sd[f"{prefix}{n}.bias"]})

    def forward_sp(self, x, mask, rng, site, B: int, S: int):
        """Sequence-parallel layer: x is this rank's [T / TP, H] token rows of the residual stream. The column-parallel
        projections read the all-gathered [T, H] (their input gradients come back reduce-scattered), the row-parallel
        products are reduce-scattered into the shard, and the bias + dropout + residual + LayerNorm run on the shard
        with the dropout mask offset to the shard's first element -- the same mask bits as the replicated layer."""
        c, tp = self.cfg, self.tp
        h, d = self.local_heads, self.head_dim
        drop = c.dropout if self.training else 0.0
        adrop = (c.dropout if c.attn_dropout is None else c.attn_dropout) if self.training else 0.0
        hip = (c.hip_gemm if c.hip_gemm is not None else os.environ.get("MIFX_BERT_HIP_GEMM", "1") == "1") and x.is_cuda
        eoff = tp.rank * x.numel()
        xg = gather_seq(x, tp)
        qkv = (hg.linear(xg, self.qkv.weight, self.qkv.bias) if hip
               else fb.linear(xg, self.qkv.weight, self.qkv.bias)).view(B, S, 3, h, d)
        if c.fused_attention:
            h0 = sum(self.heads_per_rank[:tp.rank])
            ctx = fb.attention(qkv, mask, 1.0 / d ** 0.5, adrop, rng, 1000 + site, h0, c.heads).reshape(B * S, h * d)
        else:
            q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
            amask = None if mask is None else mask[:, None, None, :].to(q.dtype)
            ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=amask, dropout_p=adrop)
            ctx = ctx.transpose(1, 2).reshape(B * S, h * d)
        a = reduce_scatter_seq(hg.linear(ctx, self.attn_out.weight) if hip else F.linear(ctx, self.attn_out.weight), tp)
        x = fb.bias_dropout_add_layernorm(a, self.attn_out.bias, x, self.ln1.weight, self.ln1.bias, c.ln_eps, drop,
                                          rng, site, eoff=eoff)
        xg = gather_seq(x, tp)
        if hip:
            o = hg.ffn(xg, self.ffn_in.weight, self.ffn_in.bias, self.ffn_out.weight)
        else:
            o = F.linear(fb.bias_gelu(F.linear(xg, self.ffn_in.weight), self.ffn_in.bias), self.ffn_out.weight)
        o = reduce_scatter_seq(o, tp)
        return fb.bias_dropout_add_layernorm(o, self.ffn_out.bias, x, self.ln2.weight, self.ln2.bias, c.ln_eps, drop,
                                             rng, site + 1, eoff=eoff)

    def sequence_parallel_params(self) -> list:
        """Parameters applied to token shards under sequence parallelism (partial gradients per rank)."""
        return [self.ln1.weight, self.ln1.bias, self.ln2.weight, self.ln2.bias, self.attn_out.bias, self.ffn_out.bias]

    def forward(self, x, mask, rng=None, site=0):
        """Dropout RNG: every mask is counter-based (model seed, step counter, site; csrc/counter_rng.h), never the
        torch generator. The hidden dropouts act on REPLICATED activations (every TP rank holds the same [B, S, H]
        tensor) and are fused with the row-parallel bias, the residual add and the LayerNorm
        (fb.bias_dropout_add_layernorm, sites `site` and `site + 1`); the attention-probability dropout indexes
        its mask by the global head (fb.attention, site 1000 + site), so both are identical for every TP split.
        (With fused_attention=False the attention dropout is SDPA's, on the torch generator.)"""
        B, S, _ = x.shape
        h, d = self.local_heads, self.head_dim
        c = self.cfg
        drop = c.dropout if self.training else 0.0
        adrop = (c.dropout if c.attn_dropout is None else c.attn_dropout) if self.training else 0.0
        # hand-written GEMM per projection only where it measured faster than hipBLASLt (mifx.ops.gemm.TUNED)
        hip = c.hip_gemm if c.hip_gemm is not None else os.environ.get("MIFX_BERT_HIP_GEMM", "1") == "1"
        hip = hip and x.is_cuda
        # (hg.linear: forward and weight gradient each on the hand-written kernel where it measured faster)
        # residual gradients folded into the input-gradient GEMMs of the projections reading the same activation
        # (hg.GradSlot: no separate gradient-sum kernel per activation); single TP rank, fused path only
        fold = (hip and self.tp.size == 1 and c.fold_residual_grad and torch.is_grad_enabled() and x.requires_grad
                and x.dtype == torch.bfloat16 and self.qkv.weight.dtype == torch.bfloat16)
        slot_a = hg.GradSlot() if fold else None
        slot_f = hg.GradSlot() if fold else None
        if hip:
            # the projection computes in the weight dtype anyway (autocast's cast of x); casting before the TP copy
            # makes its backward all-reduce a bf16 one (the peer-memory kernels: no host collective in the captured
            # step) -- the first layer's input is the fp32 embedding LayerNorm output. Cast at TP = 1 too: an fp32
            # input would send the first layer's QKV projection to the library (F.linear under autocast: weight
            # gradient, bias sum and input gradient as three aten kernels, ~100 us) instead of the hand-written
            # backward with its weight gradient in the grouped launch
            cdt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else self.qkv.weight.dtype
            xin = x if x.dtype == cdt else x.to(cdt)
            # (copy_to_tp folded into the projection: its input gradient is all-reduced, overlapped with its GEMM)
            qkv = hg.linear(xin, self.qkv.weight, self.qkv.bias, slot=slot_a, tp_in=self.tp).view(B, S, 3, h, d)
        else:
            qkv = self.qkv(x).view(B, S, 3, h, d)
        if c.fused_attention:
            # fused attention straight on the projection output (no q/k/v transposes); its dropout mask is keyed
            # by the GLOBAL head index, so it is identical for any TP split (site: this layer's attention)
            h0 = sum(self.heads_per_rank[:self.tp.rank])
            ctx = fb.attention(qkv, mask, 1.0 / d ** 0.5, adrop, rng, 1000 + site, h0, c.heads).reshape(B, S, h * d)
        else:
            # q/k/v as [B, h, S, d] views; unbind so the backward assembles dq/dk/dv with ONE stack copy
            q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
            amask = None if mask is None else mask[:, None, None, :].to(q.dtype)
            ctx = F.scaled_dot_product_attention(q, k, v, attn_mask=amask, dropout_p=adrop)
            ctx = ctx.transpose(1, 2).reshape(B, S, h * d)
        tokens = B * S
        if hip and overlap_ok(self.tp, tokens, c.hidden):  # row-parallel GEMM + all-reduce overlapped in token chunks
            a = hg.linear(ctx, self.attn_out.weight, tp=self.tp)
        elif hip:
            a = reduce_from_tp(hg.linear(ctx, self.attn_out.weight), self.tp)
        else:
            a = self.attn_out(ctx, add_bias=False)
        x = fb.bias_dropout_add_layernorm(a, self.attn_out.bias, x, self.ln1.weight, self.ln1.bias, c.ln_eps, drop,
                                          rng, site, slot=slot_a)
        if hip and overlap_ok(self.tp, tokens, c.hidden):  # (FFN-out all-reduced inside, overlapped)
            o = hg.ffn(x, self.ffn_in.weight, self.ffn_in.bias, self.ffn_out.weight, slot=slot_f, tp=self.tp,
                       tp_in=self.tp)
        elif hip:  # FFN-in + GELU + FFN-out as one autograd node (the dH GEMM and the GELU backward fused)
            o = reduce_from_tp(hg.ffn(x, self.ffn_in.weight, self.ffn_in.bias, self.ffn_out.weight, slot=slot_f,
                                      tp_in=self.tp), self.tp)
        else:
            f = fb.bias_gelu(F.linear(copy_to_tp(x, self.tp), self.ffn_in.weight), self.ffn_in.bias)
            o = self.ffn_out(f, add_bias=False)
        return fb.bias_dropout_add_layernorm(o, self.ffn_out.bias, x, self.ln2.weight, self.ln2.bias, c.ln_eps, drop,
                                             rng, site + 1, slot=slot_f)


class BertForSequenceClassification(nn.Module):
    def __init__(self, cfg: BertConfig | None = None, tp: TPGroup | None = None, seed: int | None = 0):
        super().__init__()
        self.cfg = cfg or BertConfig()
        self.tp = tp or TPGroup(None)
        c = self.cfg
        self.word = VocabParallelEmbedding(c.vocab_size, c.hidden, self.tp)
        self.pos = nn.Embedding(c.max_position, c.hidden)
        self.tok_type = nn.Embedding(c.type_vocab, c.hidden)
        self.ln_emb = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.layers = nn.ModuleList([BertLayer(c, self.tp) for _ in range(c.layers)])
        self.pooler = nn.Linear(c.hidden, c.hidden)
        self.classifier = nn.Linear(c.hidden, c.num_labels)
        # hidden-dropout RNG state [seed, step counter] (device int64; advanced in-graph once per training forward)
        self.register_buffer("drop_rng", torch.tensor([c.dropout_seed, 0], dtype=torch.int64), persistent=False)
        if seed is not None:
            self.init_weights(seed)

    @property
    def sequence_parallel(self) -> bool:
        return self.cfg.sequence_parallel and self.tp.size > 1

    def sync_sequence_parallel_grads(self) -> None:
        """After the backward, before the update: sum the token-shard parameters' gradients over the TP group
        (no-op without sequence parallelism). Once per optimizer step, after the last micro-batch's backward: the
        sum is over whatever the gradients hold."""
        if self.sequence_parallel:
            all_reduce_grads([p for L in self.layers for p in L.sequence_parallel_params()], self.tp)

    def init_weights(self, seed: int) -> None:
        """Initialise as the full model would, then take this rank's shard (so any TP degree matches TP=1)."""
        full = full_init_state(self.cfg, seed)
        self.load_full(full)

    def load_full(self, sd: dict) -> None:
        self.word.load_full(sd["word.weight"])
        for n in ("pos", "tok_type", "ln_emb", "pooler", "classifier"):
            getattr(self, n).load_state_dict({k.split(".", 1)[1]: v for k, v in sd.items() if k.startswith(n + ".")})
        for i, layer in enumerate(self.layers):
            layer.load_full(sd, f"layers.{i}.")

    def forward(self, input_ids, token_type_ids=None, attention_mask=None):
        B, S = input_ids.shape
        pos = torch.arange(S, device=input_ids.device)
        tt = token_type_ids if token_type_ids is not None else torch.zeros_like(input_ids)
        drop = self.cfg.dropout if self.training else 0.0
        rng = self.drop_rng
        if drop > 0:
            self.drop_rng[1:].add_(1)  # new masks every step (captured into the step's hipGraph)
            rng = fb.rng_snapshot(self.drop_rng)  # this forward's state, shared by all its dropout sites
        a = self.word(input_ids) + fb.embedding(pos, self.pos.weight)[None]
        te = fb.embedding(tt, self.tok_type.weight)
        if a.is_cuda and a.dtype == torch.bfloat16 and te.dtype == a.dtype and self.tp.size == 1:
            # LayerNorm(word + position + token type) as the fused add + LayerNorm kernel (bf16 out, fp32 inside): no
            # fp32 activation and no library LayerNorm forward / backward with its casts (~40 us per step). TP = 1
            # (the measured configuration) only: TP > 1 keeps the path its multi-rank rehearsals were validated on
            # (the 8-rank shared-GPU sequence-parallel test timed out twice with it, cause not isolated in round 6)
            x = fb.add_layernorm(a, te, self.ln_emb.weight, self.ln_emb.bias, self.ln_emb.eps)
        else:
            x = self.ln_emb(a + te)
        x = fb.dropout(x, drop, rng, 0)
        mask = None
        if attention_mask is not None:  # additive key bias [B, S] (fp32; -1e30 on padding keys)
            mask = ((1.0 - attention_mask.float()) * -1e30).contiguous()
        sp = self.sequence_parallel
        if sp and (B * S) % self.tp.size:
            if self.training and torch.is_grad_enabled():
                raise ValueError(f"sequence parallelism: {B} x {S} tokens do not split over {self.tp.size} ranks")
            sp = False  # (inference on an odd-sized batch: the replicated layers compute the same function)
        if sp:
            # the layers' residual stream: this rank's token rows, in the dtype the projections compute in
            cdt = torch.get_autocast_dtype("cuda") if x.is_cuda and torch.is_autocast_enabled("cuda") else x.dtype
            x = scatter_to_seq(x.reshape(B * S, -1), self.tp, cdt)
            for i, layer in enumerate(self.layers):
                x = layer.forward_sp(x, mask, rng, 1 + 2 * i, B, S)
            x = gather_seq_replicated(x, self.tp).view(B, S, -1)
        else:
            for i, layer in enumerate(self.layers):
                x = layer(x, mask, rng, 1 + 2 * i)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        return self.classifier(fb.dropout(pooled, drop, rng, 1 + 2 * len(self.layers)))


def full_init_state(cfg: BertConfig, seed: int) -> dict:
    """TP=1 parameter dict (BERT init: N(0, 0.02) weights, zero biases, unit LayerNorm)."""
    g = torch.Generator().manual_seed(seed)

    def n(*shape):
        return torch.randn(*shape, generator=g) * cfg.init_std

    H, I = cfg.hidden, cfg.intermediate
    sd = {"word.weight": n(cfg.vocab_size, H), "pos.weight": n(cfg.max_position, H), "tok_type.weight": n(cfg.type_vocab, H),
          "ln_emb.weight": torch.ones(H), "ln_emb.bias": torch.zeros(H), "pooler.weight": n(H, H),
          "pooler.bias": torch.zeros(H), "classifier.weight": n(cfg.num_labels, H),
          "classifier.bias": torch.zeros(cfg.num_labels)}
    for i in range(cfg.layers):
        p = f"layers.{i}."
        sd.update({p + "qkv.weight": n(3 * H, H), p + "qkv.bias": torch.zeros(3 * H),
                   p + "attn_out.weight": n(H, H), p + "attn_out.bias": torch.zeros(H),
                   p + "ln1.weight": torch.ones(H), p + "ln1.bias": torch.zeros(H),
                   p + "ffn_in.weight": n(I, H), p + "ffn_in.bias": torch.zeros(I),
                   p + "ffn_out.weight": n(H, I), p + "ffn_out.bias": torch.zeros(H),
                   p + "ln2.weight": torch.ones(H), p + "ln2.bias": torch.zeros(H)})
    return sd


def gather_full_state(model: BertForSequenceClassification) -> dict:
    """Reassemble the TP=1 state dict from all ranks (for checkpoints / equivalence tests)."""
    import torch.distributed as dist

    tp = model.tp

    def gather(t: torch.Tensor, dim: int, sizes) -> torch.Tensor:
        if tp.size == 1:
            return t.detach().clone()
        mx = max(sizes)
        pad = [0, 0] * (t.dim() - 1 - dim) + [0, mx - t.shape[dim]]
        tt = F.pad(t.detach(), pad).contiguous()
        outs = [torch.empty_like(tt) for _ in range(tp.size)]
        dist.all_gather(outs, tt, group=tp.group)
        return torch.cat([o.narrow(dim, 0, s) for o, s in zip(outs, sizes)], dim)

    sd = {"word.weight": gather(model.word.weight, 0, model.word.sizes)}
    for n in ("pos", "tok_type", "ln_emb", "pooler", "classifier"):
        for k, v in getattr(model, n).state_dict().items():
            sd[f"{n}.{k}"] = v.detach().clone()
    for i, L in enumerate(model.layers):
        p = f"layers.{i}."
        d = L.head_dim
        w = gather(L.qkv.weight, 0, L.qkv.sizes)
        b = gather(L.qkv.bias, 0, L.qkv.sizes)
        # re-interleave per-rank [q_r; k_r; v_r] blocks into [Q; K; V]
        chunks_w, chunks_b, off = [[], [], []], [[], [], []], 0
        for h in L.heads_per_rank:
            for k in range(3):
                chunks_w[k].append(w[off + k * h * d: off + (k + 1) * h * d])
                chunks_b[k].append(b[off + k * h * d: off + (k + 1) * h * d])
            off += 3 * h * d
        sd[p + "qkv.weight"] = torch.cat([torch.cat(c) for c in chunks_w])
        sd[p + "qkv.bias"] = torch.cat([torch.cat(c) for c in chunks_b])
        sd[p + "attn_out.weight"] = gather(L.attn_out.weight, 1, L.attn_out.sizes)
        sd[p + "attn_out.bias"] = L.attn_out.bias.detach().clone()
        sd[p + "ffn_in.weight"] = gather(L.ffn_in.weight, 0, L.ffn_in.sizes)
        sd[p + "ffn_in.bias"] = gather(L.ffn_in.bias, 0, L.ffn_in.sizes)
        sd[p + "ffn_out.weight"] = gather(L.ffn_out.weight, 1, L.ffn_out.sizes)
        sd[p + "ffn_out.bias"] = L.ffn_out.bias.detach().clone()
        for n in ("ln1", "ln2"):
            sd[f"{p}{n}.weight"] = getattr(L, n).weight.detach().clone()
            sd[f"{p}{n}.bias"] = getattr(L, n).bias.detach().clone()
    return sd


def num_params(cfg: BertConfig) -> int:
    H, I, L = cfg.hidden, cfg.intermediate, cfg.layers
    per_layer = 3 * H * H + 3 * H + H * H + H + 2 * H + I * H + I + H * I + H + 2 * H
    return (cfg.vocab_size + cfg.max_position + cfg.type_vocab) * H + 2 * H + L * per_layer + H * H + H \
        + cfg.num_labels * (H + 1)
