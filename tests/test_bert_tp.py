"""BERT + Megatron-style tensor parallelism: TP=2/3 (gloo, CPU) must equal the TP=1 model exactly
(uneven head split at TP=3), for the forward logits and for parameters after an optimizer step."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mifx.models.bert import BertConfig, BertForSequenceClassification, full_init_state, gather_full_state, num_params
from mifx.ops import fused_bert as fb_mod
from mifx.parallel.tensor_parallel import TPGroup, head_partition, split_sizes


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(cfg, B=3, S=16, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, cfg.vocab_size, (B, S), generator=g)
    tt = torch.randint(0, 2, (B, S), generator=g)
    am = torch.ones(B, S)
    am[0, 12:] = 0
    y = torch.randint(0, cfg.num_labels, (B,), generator=g)
    return ids, tt, am, y


def _step(model, cfg, lr=0.1):
    ids, tt, am, y = _batch(cfg)
    model.zero_grad(set_to_none=True)
    logits = model(ids, tt, am)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    model.sync_sequence_parallel_grads()  # (sequence parallelism: token-shard parameters' partial gradients)
    with torch.no_grad():
        for p in model.parameters():
            p -= lr * p.grad
    return logits.detach()


def _worker(rank, world, port, out, cfg_kw=None, steps=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = BertConfig.tiny(**(cfg_kw or {"dropout": 0.0}))
    torch.manual_seed(100 + rank)  # per-rank torch generator streams: replicated dropout must not depend on them
    m = BertForSequenceClassification(cfg, TPGroup(), seed=1)
    for _ in range(steps):
        logits = _step(m, cfg)
    full = gather_full_state(m)
    # replicated parameters (LayerNorms, row-parallel biases, pos / token-type embeddings, pooler, classifier)
    # as this rank holds them, to check they stayed bit-identical across the TP ranks
    repl = {n: p.detach().clone() for n, p in m.named_parameters()
            if not any(s in n for s in ("qkv.", "ffn_in.", "word.")) and not n.endswith(("attn_out.weight",
                                                                                            "ffn_out.weight"))}
    torch.save(repl, f"{out}.repl{rank}")
    if rank == 0:
        torch.save({"logits": logits, "state": full}, out)
    dist.destroy_process_group()


def test_partitions():
    assert head_partition(12, 8) == [2, 2, 2, 2, 1, 1, 1, 1]
    assert split_sizes(3072, 8) == [384] * 8 and sum(split_sizes(30522, 8)) == 30522
    assert num_params(BertConfig()) == sum(v.numel() for v in full_init_state(BertConfig(layers=1), 0).values()) \
        + 11 * (sum(v.numel() for k, v in full_init_state(BertConfig(layers=1), 0).items() if k.startswith("layers.")))


@pytest.mark.parametrize("world", [2, 3])
def test_tp_matches_single_process(world):
    cfg = BertConfig.tiny(dropout=0.0)
    ref = BertForSequenceClassification(cfg, None, seed=1)
    ref_logits = _step(ref, cfg)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, start_method="spawn")
        got = torch.load(out, weights_only=True)
    torch.testing.assert_close(got["logits"], ref_logits, rtol=1e-5, atol=1e-5)
    ref_sd = gather_full_state(ref)
    for k, v in ref_sd.items():
        np.testing.assert_allclose(got["state"][k].numpy(), v.numpy(), rtol=1e-4, atol=1e-6, err_msg=k)


def test_tp_dropout_replicated_params_identical_and_match_tp1():
    """Hidden dropout > 0 at TP=2 (gloo): the replicated activations' masks are keyed by (seed, step, site), not by
    each rank's torch generator, so (a) replicated parameters stay bit-identical across ranks over several steps
    and (b) with attention-probability dropout off the TP=2 trajectory equals TP=1 (same masks)."""
    kw = {"dropout": 0.1, "attn_dropout": 0.0}
    cfg = BertConfig.tiny(**kw)
    ref = BertForSequenceClassification(cfg, None, seed=1)
    for _ in range(3):
        ref_logits = _step(ref, cfg)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(2, _port(), out, kw, 3), nprocs=2, start_method="spawn")
        got = torch.load(out, weights_only=True)
        r0 = torch.load(f"{out}.repl0", weights_only=True)
        r1 = torch.load(f"{out}.repl1", weights_only=True)
    assert len(r0) > 10 and r0.keys() == r1.keys()
    for k in r0:
        assert torch.equal(r0[k], r1[k]), f"replicated parameter {k} diverged across TP ranks"
    torch.testing.assert_close(got["logits"], ref_logits, rtol=1e-4, atol=1e-5)
    for k, v in gather_full_state(ref).items():
        np.testing.assert_allclose(got["state"][k].numpy(), v.numpy(), rtol=1e-3, atol=1e-5, err_msg=k)


def test_tp_attention_dropout_keeps_replicated_params_identical():
    """With attention-probability dropout on too (uneven head split at TP=3): its mask is indexed by the GLOBAL
    head, so replicated parameters stay bit-identical across ranks AND the TP=3 trajectory equals TP=1."""
    cfg = BertConfig.tiny(dropout=0.1)
    ref = BertForSequenceClassification(cfg, None, seed=1)
    for _ in range(2):
        ref_logits = _step(ref, cfg)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(3, _port(), out, {"dropout": 0.1}, 2), nprocs=3, start_method="spawn")
        reps = [torch.load(f"{out}.repl{r}", weights_only=True) for r in range(3)]
        got = torch.load(out, weights_only=True)
    for k in reps[0]:
        assert torch.equal(reps[0][k], reps[1][k]) and torch.equal(reps[0][k], reps[2][k]), k
    torch.testing.assert_close(got["logits"], ref_logits, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("world", [2, 3])
def test_sequence_parallel_matches_tp1_and_keeps_replicas_identical(world):
    """Sequence parallelism (residual stream, LayerNorms and hidden dropouts on each rank's 1/TP of the tokens;
    reduce-scatter / all-gather instead of all-reduces; token-shard parameter gradients summed over the group) with
    hidden AND attention dropout on, uneven heads at TP=3: the trajectory equals TP=1 (the shard's dropout mask is
    the replicated mask offset to the shard) and the replicated parameters stay bit-identical across ranks."""
    kw = {"dropout": 0.1, "sequence_parallel": True}
    cfg = BertConfig.tiny(**kw)
    ref = BertForSequenceClassification(cfg, None, seed=1)
    assert not ref.sequence_parallel  # (TP = 1: the plain layer)
    for _ in range(2):
        ref_logits = _step(ref, cfg)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.start_processes(_worker, args=(world, _port(), out, kw, 2), nprocs=world, start_method="spawn")
        reps = [torch.load(f"{out}.repl{r}", weights_only=True) for r in range(world)]
        got = torch.load(out, weights_only=True)
    for r in range(1, world):
        for k in reps[0]:
            assert torch.equal(reps[0][k], reps[r][k]), k
    torch.testing.assert_close(got["logits"], ref_logits, rtol=1e-4, atol=1e-5)
    for k, v in gather_full_state(ref).items():
        np.testing.assert_allclose(got["state"][k].numpy(), v.numpy(), rtol=1e-3, atol=1e-5, err_msg=k)


def test_sequence_parallel_needs_divisible_tokens():
    from mifx.parallel.tensor_parallel import _seq_rows

    class _G:
        size = 3

    assert _seq_rows(48, _G()) == 16
    with pytest.raises(ValueError):
        _seq_rows(47, _G())


def test_attention_reference_matches_sdpa_and_masks():
    from mifx.ops import fused_bert as fb

    torch.manual_seed(4)
    B, S, H, Dh = 2, 16, 3, 8
    qkv = torch.randn(B, S, 3, H, Dh)
    am = torch.ones(B, S)
    am[1, 11:] = 0
    kb = (1.0 - am) * -1e30
    got = fb.attention(qkv, kb, Dh ** -0.5)
    q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=(kb[:, None, None, :] > -1))
    torch.testing.assert_close(got, ref.transpose(1, 2), rtol=1e-5, atol=1e-5)
    rng = torch.tensor([3, 9])
    d1 = fb.attention(qkv, kb, Dh ** -0.5, 0.2, rng, 7)
    assert not torch.allclose(d1, got)
    # a head slice with its global offset draws the same mask as the full model (TP invariance)
    part = fb.attention(qkv[:, :, :, 1:3].contiguous(), kb, Dh ** -0.5, 0.2, rng, 7, h0=1, htot=3)
    torch.testing.assert_close(part, d1[:, :, 1:3])


def test_counter_dropout_mask_cpu():
    from mifx.ops import fused_bert as fb

    rng = torch.tensor([7, 3], dtype=torch.int64)
    m = fb.keep_mask(100_003, rng, 5, 0.1)
    assert abs(1 - m.float().mean().item() - 0.1) < 0.005
    assert torch.equal(m, fb.keep_mask(100_003, rng, 5, 0.1))  # deterministic
    assert not torch.equal(m, fb.keep_mask(100_003, rng, 6, 0.1))  # per site
    assert not torch.equal(m, fb.keep_mask(100_003, torch.tensor([7, 4]), 5, 0.1))  # per step
    a, r = torch.randn(6, 32), torch.randn(6, 32)
    bias, w, b = torch.randn(32), torch.randn(32), torch.randn(32)
    y = fb.bias_dropout_add_layernorm(a, bias, r, w, b, 1e-5, 0.25, rng, 2)
    keep = fb.keep_mask(a.numel(), rng, 2, 0.25).view(6, 32)
    ref = torch.nn.functional.layer_norm(torch.where(keep, (a + bias) / 0.75, 0.0) + r, (32,), w, b, 1e-5)
    torch.testing.assert_close(y, ref)
    x = torch.randn(5, 9)
    torch.testing.assert_close(fb.dropout(x, 0.5, rng, 1), torch.where(fb.keep_mask(45, rng, 1, 0.5).view(5, 9),
                                                                      x * 2, 0.0))


@pytest.mark.gpu
@pytest.mark.parametrize("S,H", [(128, 12), (64, 5), (192, 3), (256, 4), (384, 3), (512, 2)])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_fused_attention_gpu(S, H, p):
    """csrc/attention.hip forward/backward against the fp32 PyTorch reference with the same key mask and the same
    counter-based dropout mask (h0 / Htot: a TP shard of a larger head set). S > 128: the chunked kernels (online
    softmax forward, dQ and dK/dV backward passes; 192 leaves half of the last 128-query block idle)."""
    from mifx.ops import native_stats
    from mifx.ops import fused_bert as fb

    torch.manual_seed(S + H)
    B, Dh, h0, htot = 3, 64, 2, H + 4
    qkv = (torch.randn(B, S, 3, H, Dh, device="cuda") * 0.7).bfloat16().requires_grad_()
    am = torch.ones(B, S, device="cuda")
    am[1, S - 9:] = 0
    am[2, S // 2:] = 0
    kb = ((1.0 - am) * -1e30).contiguous()
    rng = torch.tensor([5, 17], dtype=torch.int64, device="cuda")
    native_stats.reset()
    out = fb.attention(qkv, kb, Dh ** -0.5, p, rng, 3, h0, htot)
    assert native_stats.snapshot()["attention"] == {"native": 1, "fallback": 0}  # the HIP kernel ran
    q32 = qkv.detach().float().requires_grad_()
    ref = fb.attention_reference(q32, kb, Dh ** -0.5, p, rng, 3, h0, htot)
    torch.testing.assert_close(out.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ref)
    out.backward(g.bfloat16())
    ref.backward(g)
    got, want = qkv.grad.float(), q32.grad
    for i, name in enumerate("qkv"):
        err = (got[:, :, i] - want[:, :, i]).norm() / want[:, :, i].norm()
        assert err < 2e-2, f"d{name}: relative error {err:.4f}"


@pytest.mark.gpu
def test_fused_bias_dropout_add_layernorm_gpu():
    """HIP fused bias + dropout + residual + LayerNorm (fwd/bwd) and standalone dropout against the CPU
    composition with the same counter-based mask (bit-identical keep pattern), fp32 / bf16, vectorised and
    scalar H."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(3)
    rng = torch.tensor([11, 5], dtype=torch.int64, device="cuda")
    for dtype, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-2)):
        for H in (64, 768, 1000):
            a = torch.randn(29, 3, H, device="cuda", dtype=dtype, requires_grad=True)
            r = torch.randn(29, 3, H, device="cuda", dtype=dtype, requires_grad=True)
            bias, w, b = (torch.randn(H, device="cuda", requires_grad=True) for _ in range(3))
            y = fb.bias_dropout_add_layernorm(a, bias, r, w, b, 1e-12, 0.1, rng, 4)
            keep = fb.keep_mask(a.numel(), rng, 4, 0.1).cuda().view(a.shape)
            a2, r2 = a.detach().float().requires_grad_(), r.detach().float().requires_grad_()
            bias2, w2, b2 = (t.detach().clone().requires_grad_() for t in (bias, w, b))
            ref = torch.nn.functional.layer_norm(torch.where(keep, (a2 + bias2) * fb._drop_scale(0.1), 0.0) + r2,
                                                 (H,), w2, b2, 1e-12)
            torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
            g = torch.randn_like(ref)
            y.backward(g.to(dtype))
            ref.backward(g)
            assert torch.equal(a.grad == 0, ~keep) or dtype == torch.bfloat16  # dropped elements get no gradient
            for got, want, sc in ((a.grad, a2.grad, 4), (r.grad, r2.grad, 4), (w.grad, w2.grad, 40),
                                  (b.grad, b2.grad, 40), (bias.grad, bias2.grad, 40)):
                torch.testing.assert_close(got.float(), want, rtol=tol * 4, atol=tol * sc)
        x = torch.randn(1001, 7, device="cuda", dtype=dtype, requires_grad=True)
        y = fb.dropout(x, 0.3, rng, 9)
        keep = fb.keep_mask(x.numel(), rng, 9, 0.3).cuda().view(x.shape)
        torch.testing.assert_close(y, torch.where(keep, x * fb._drop_scale(0.3), 0.0).to(dtype))
        y.backward(torch.ones_like(y))
        torch.testing.assert_close(x.grad, torch.where(keep, fb._drop_scale(0.3), 0.0).to(dtype))


@pytest.mark.gpu
def test_fused_add_layernorm_and_bias_gelu_gpu():
    from mifx.ops import fused_bert as fb

    torch.manual_seed(0)
    for dtype, tol in ((torch.float32, 1e-5), (torch.bfloat16, 2e-2)):
        for H in (64, 256, 768, 1000, 1024):  # 256/768/1024: vectorised paths; 64/1000: scalar
            a = torch.randn(37, 5, H, device="cuda", dtype=dtype, requires_grad=True)
            r = torch.randn(37, 5, H, device="cuda", dtype=dtype, requires_grad=True)
            w = torch.randn(H, device="cuda", requires_grad=True)
            b = torch.randn(H, device="cuda", requires_grad=True)
            y = fb.add_layernorm(a, r, w, b, 1e-12)
            a32, r32 = a.detach().float().requires_grad_(), r.detach().float().requires_grad_()
            w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
            ref = torch.nn.functional.layer_norm(a32 + r32, (H,), w2, b2, 1e-12)
            torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
            g = torch.randn_like(ref)
            y.backward(g.to(dtype))
            ref.backward(g)
            torch.testing.assert_close(a.grad.float(), a32.grad, rtol=tol * 4, atol=tol * 4)
            torch.testing.assert_close(w.grad, w2.grad, rtol=tol * 4, atol=tol * 40)
            torch.testing.assert_close(b.grad, b2.grad, rtol=tol * 4, atol=tol * 40)
        for M, N in ((64, 3072), (1000, 3072), (70, 3070)):  # last: scalar fallback (N % 8 != 0)
            x = torch.randn(M, N, device="cuda", dtype=dtype, requires_grad=True)
            bias = torch.randn(N, device="cuda", requires_grad=True)
            y = fb.bias_gelu(x, bias)
            x2, b2 = x.detach().float().requires_grad_(), bias.detach().clone().requires_grad_()
            ref = torch.nn.functional.gelu(x2 + b2)
            torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
            g = torch.randn_like(ref)
            y.backward(g.to(dtype))
            ref.backward(g)
            torch.testing.assert_close(x.grad.float(), x2.grad, rtol=tol * 4, atol=tol * 4)
            torch.testing.assert_close(bias.grad, b2.grad, rtol=tol * 4, atol=tol * 60)


@pytest.mark.gpu
def test_fused_add_layernorm_many_rows_per_wave():
    """More rows than waves (R > 8 x 1024: each wave of the backward walks several row pairs, the last one odd)
    against the fp32 composition."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(4)
    H = 768
    a = torch.randn(9001, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    r = torch.randn(9001, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(H, device="cuda", requires_grad=True)
    b = torch.randn(H, device="cuda", requires_grad=True)
    y = fb.add_layernorm(a, r, w, b, 1e-12)
    a32, r32 = a.detach().float().requires_grad_(), r.detach().float().requires_grad_()
    w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    ref = torch.nn.functional.layer_norm(a32 + r32, (H,), w2, b2, 1e-12)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ref)
    y.backward(g.to(torch.bfloat16))
    ref.backward(g)
    torch.testing.assert_close(a.grad.float(), a32.grad, rtol=8e-2, atol=8e-2)
    torch.testing.assert_close(w.grad, w2.grad, rtol=8e-2, atol=0.05 * float(w2.grad.abs().max()))
    torch.testing.assert_close(b.grad, b2.grad, rtol=8e-2, atol=0.05 * float(b2.grad.abs().max()))


@pytest.mark.gpu
def test_fused_ln_gelu_bf16_parameters():
    """bf16 model (FlatAdamW): gamma/beta/bias are read as bf16 and dw/db/dbias written as bf16 by the kernels
    (no cast kernels); compared with an fp32 PyTorch reference of the same bf16-rounded parameters."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(1)
    for H in (768, 1000):  # vectorised / scalar LayerNorm paths
        a = torch.randn(64, 3, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        r = torch.randn(64, 3, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        b = torch.randn(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        y = fb.add_layernorm(a, r, w, b, 1e-12)
        a32, r32 = a.detach().float().requires_grad_(), r.detach().float().requires_grad_()
        w2, b2 = w.detach().float().requires_grad_(), b.detach().float().requires_grad_()
        ref = torch.nn.functional.layer_norm(a32 + r32, (H,), w2, b2, 1e-12)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        g = torch.randn_like(ref)
        y.backward(g.bfloat16())
        ref.backward(g)
        assert w.grad.dtype == b.grad.dtype == torch.bfloat16
        torch.testing.assert_close(w.grad.float(), w2.grad, rtol=3e-2, atol=0.5)
        torch.testing.assert_close(b.grad.float(), b2.grad, rtol=3e-2, atol=0.5)
    for M, N in ((256, 3072), (70, 3070)):
        x = torch.randn(M, N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        bias = torch.randn(N, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        y = fb.bias_gelu(x, bias)
        x2, b2 = x.detach().float().requires_grad_(), bias.detach().float().requires_grad_()
        ref = torch.nn.functional.gelu(x2 + b2)
        torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
        g = torch.randn_like(ref)
        y.backward(g.bfloat16())
        ref.backward(g)
        assert bias.grad.dtype == torch.bfloat16
        torch.testing.assert_close(bias.grad.float(), b2.grad, rtol=3e-2, atol=0.5)


@pytest.mark.gpu
def test_linear_and_bias_add_bias_grad_kernels():
    """fb.linear / fb.bias_add (bias gradient by the deterministic HIP column sum) against F.linear / add,
    fp32 and bf16 parameters, with and without autocast."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(2)
    for pdt, amp in ((torch.float32, False), (torch.float32, True), (torch.bfloat16, True)):
        for M, K, N in ((4096, 768, 2304), (70, 64, 3070)):
            x = torch.randn(M, K, device="cuda", dtype=pdt, requires_grad=True)
            w = (torch.randn(N, K, device="cuda") * 0.05).to(pdt).requires_grad_()
            b = torch.randn(N, device="cuda", dtype=pdt, requires_grad=True)
            x2, w2, b2 = (t.detach().clone().requires_grad_() for t in (x, w, b))
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                y = fb.bias_add(fb.linear(x, w, b), b)
                ref = torch.nn.functional.linear(x2, w2, b2)
                ref = ref + b2.to(ref.dtype)
            assert y.dtype == ref.dtype
            g = torch.randn_like(ref)
            y.backward(g)
            ref.backward(g)
            tol = 2e-2 if (amp or pdt == torch.bfloat16) else 1e-4
            torch.testing.assert_close(y.float(), ref.float(), rtol=tol, atol=tol)
            for a, r in ((x.grad, x2.grad), (w.grad, w2.grad)):
                assert a.dtype == r.dtype
                torch.testing.assert_close(a.float(), r.float(), rtol=tol, atol=tol * 10)
            assert b.grad.dtype == pdt
            gs = g.float().sum(0)
            torch.testing.assert_close(b.grad.float(), 2 * gs, rtol=tol, atol=tol * 50)


@pytest.mark.gpu
def test_bert_base_gpu_train_step_bf16():
    cfg = BertConfig(dropout=0.0)
    m = BertForSequenceClassification(cfg, None, seed=0).cuda()
    ids, tt, am, y = (t.cuda() for t in _batch(cfg, B=8, S=128))
    opt = torch.optim.AdamW(m.parameters(), lr=2e-5, fused=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = torch.nn.functional.cross_entropy(m(ids, tt, am).float(), y)
    loss.backward()
    opt.step()
    assert torch.isfinite(loss)


@pytest.mark.gpu
def test_bert_hipgraph_step_matches_eager():
    from mifx.trainer.bert_trainer import BertTrainer

    cfg = BertConfig(layers=2, dropout=0.0)
    eager = BertTrainer(cfg, 8, 64, "cuda", graph=False, flat_adamw=False)
    graphed = BertTrainer(cfg, 8, 64, "cuda", graph=True, flat_adamw=False)
    le = [float(eager.step()) for _ in range(6)]
    lg = [float(graphed.step()) for _ in range(3)]  # capture runs 3 eager warmup steps first
    assert graphed.graph is not None
    np.testing.assert_allclose(lg, le[3:], rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_bert_hipgraph_flat_adamw_matches_eager_flat_adamw():
    """The default configuration (hipGraph + FlatAdamW reading autograd's own gradients) against the same
    optimizer stepped eagerly, over 12 steps of a 2-layer model with dropout off."""
    from mifx.trainer.bert_trainer import BertTrainer

    cfg = BertConfig(layers=2, dropout=0.0)
    eager = BertTrainer(cfg, 8, 64, "cuda", graph=False)
    graphed = BertTrainer(cfg, 8, 64, "cuda", graph=True)
    assert eager.flat and graphed.flat and graphed.use_graph
    le = [float(eager.step()) for _ in range(15)]
    lg = [float(graphed.step()) for _ in range(12)]  # capture runs 3 eager warmup steps first
    np.testing.assert_allclose(lg, le[3:], rtol=2e-2, atol=2e-3)


@pytest.mark.gpu
def test_bert_trainer_main_default_config_stays_finite(capsys):
    """Regression: the default 12-layer B=32 S=128 configuration of bert_trainer.main (hipGraph replay) must
    keep a finite loss over its timed steps (before the scatter-add embedding backward, the captured step went
    non-finite after ~10 replays: rocPRIM's partition kernel in PyTorch's embedding backward faults under
    graph replay)."""
    import json

    from mifx.trainer.bert_trainer import main

    main(["--steps", "15", "--warmup", "5"])
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out["hipgraph"] is True
    assert np.isfinite(out["loss"]), out
    assert out["value"] > 0


@pytest.mark.gpu
def test_bert_seq256_dropout_hipgraph_stays_finite():
    """S=256 is outside the fused attention kernel's shapes: with dropout on, the fallback draws its mask on the
    device (no host sync), so the whole step still captures into a hipGraph (regression: the host mask broke
    capture)."""
    from mifx.trainer.bert_trainer import BertTrainer

    cfg = BertConfig(layers=2, dropout=0.1)
    tr = BertTrainer(cfg, 4, 256, "cuda", graph=True)
    losses = [float(tr.step()) for _ in range(4)]
    assert tr.graph is not None
    assert all(np.isfinite(losses)), losses


@pytest.mark.gpu
def test_attention_fallback_device_mask_matches_host_mask():
    import mifx.ops.fused_bert as fb

    rng = torch.tensor([7, 3], dtype=torch.int64, device="cuda")
    dev = fb.device_keep_mask(4 * 2 * 256 * 256, rng, 1005, 0.1, torch.device("cuda")).cpu()
    host = fb.keep_mask(4 * 2 * 256 * 256, rng, 1005, 0.1)
    assert torch.equal(dev, host)


@pytest.mark.gpu
def test_dropout_backward_uses_forward_time_rng_snapshot():
    """Advancing the live counter between forward and backward must not change the backward's mask."""
    import mifx.ops.fused_bert as fb

    x = torch.randn(64, 256, device="cuda", requires_grad=True)
    rng = torch.tensor([11, 0], dtype=torch.int64, device="cuda")
    y = fb.dropout(x, 0.3, rng, 2)
    rng[1:].add_(5)  # e.g. a second training forward before this backward
    y.backward(torch.ones_like(y))
    keep = (y.detach() != 0).float()
    torch.testing.assert_close(x.grad, keep / 0.7, rtol=1e-6, atol=1e-6)


def test_rng_snapshot_shared_by_the_sites_of_one_forward():
    """One frozen [seed, counter] snapshot per model forward: every dropout site keeps that tensor (no per-site copy),
    a live (mutable) state tensor is still copied at forward time, and advancing the live counter afterwards does not
    change what the snapshot holds (the masks recomputed in backward stay the forward's)."""
    from mifx.ops import fused_bert as fb

    live = torch.tensor([1234, 7], dtype=torch.int64)
    snap = fb.rng_snapshot(live)
    assert fb._snap(snap, 0.1) is snap
    copy = fb._snap(live, 0.1)
    assert copy is not live and torch.equal(copy, live)
    assert fb._snap(live, 0.0) is None and fb._snap(None, 0.1) is None
    live[1:].add_(1)
    assert int(snap[1]) == 7 and int(copy[1]) == 7


def test_model_forward_uses_one_snapshot_per_step():
    cfg = BertConfig.tiny(dropout=0.1)
    m = BertForSequenceClassification(cfg, seed=0)
    m.train()
    ids = torch.randint(0, cfg.vocab_size, (2, 8))
    seen = []
    orig = fb_mod.dropout

    def spy(x, p, rng, site):
        seen.append(rng)
        return orig(x, p, rng, site)

    fb_mod.dropout = spy
    try:
        m(ids)
    finally:
        fb_mod.dropout = orig
    assert len(seen) == 2 and seen[0] is seen[1] and getattr(seen[0], "_mifx_frozen", False)
    assert int(seen[0][1]) == int(m.drop_rng[1]) == 1


def test_grad_slot_folds_residual_gradient_into_dx():
    """hg.GradSlot: the residual gradient parked by the add+LayerNorm backward is added by the projection's dX GEMM
    (one addmm), and an empty slot fails loudly instead of dropping the residual gradient."""
    from mifx.ops import gemm as hg

    torch.manual_seed(0)
    x = torch.randn(6, 5, 16, requires_grad=True)
    w = torch.randn(24, 16, requires_grad=True)
    G, R = torch.randn(6, 5, 24), torch.randn(6, 5, 16)
    slot = hg.GradSlot()
    y = hg.linear(x, w, slot=slot)
    slot.g = R
    (y * G).sum().backward()
    torch.testing.assert_close(x.grad, G @ w.detach() + R)
    torch.testing.assert_close(w.grad, G.reshape(-1, 24).t() @ x.detach().reshape(-1, 16))
    assert slot.g is None
    y = hg.linear(x, w, slot=hg.GradSlot())
    with pytest.raises(RuntimeError, match="GradSlot empty"):
        y.sum().backward()


@pytest.mark.gpu
def test_bert_residual_grad_fold_matches_autograd_sum():
    """A bf16 BERT layer stack with the residual gradients folded into the dX GEMMs (default) against autograd's
    own gradient sums (fold_residual_grad=False): same loss, every parameter gradient within bf16 rounding."""
    grads = {}
    for fold in (True, False):
        cfg = BertConfig(layers=2, dropout=0.0, fold_residual_grad=fold)
        m = BertForSequenceClassification(cfg, None, seed=0).cuda().to(torch.bfloat16)
        ids, tt, am, y = (t.cuda() for t in _batch(cfg, B=8, S=128))
        loss = torch.nn.functional.cross_entropy(m(ids, tt, am).float(), y)
        loss.backward()
        grads[fold] = (float(loss), {n: p.grad.float() for n, p in m.named_parameters() if p.grad is not None})
    (l1, g1), (l0, g0) = grads[True], grads[False]
    assert l1 == l0
    assert g1.keys() == g0.keys()
    for n in g0:
        err = (g1[n] - g0[n]).abs().max().item() / max(g0[n].abs().max().item(), 1e-6)
        assert err < 3e-2, (n, err)


@pytest.mark.gpu
def test_embedding_backward_deterministic_gpu():
    """mifx.ops.fused_bert.embedding's backward (csrc/fused_bert.hip emb_bwd_chunks / emb_bwd_combine: an id's rows
    summed in token order, chunks of 64 occurrences on separate workgroups added in chunk order) equals the fp64
    scatter-add and is bit-identical run to run: repeated position ids (32 each), random token ids, token-type ids
    (2048 occurrences each: 32 chunks), a mostly-one-id batch, on the vector (bf16 H 768, fp32 H 96) and scalar
    (H 100) column paths."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(21)
    skew = torch.randint(0, 50, (5000,), device="cuda")
    skew[torch.rand(5000, device="cuda") < 0.9] = 3
    cases = [(torch.arange(128, device="cuda").repeat(32), 96, torch.bfloat16),
             (torch.randint(0, 3000, (4096,), device="cuda"), 96, torch.bfloat16),
             (torch.arange(4096, device="cuda") // 2048, 768, torch.bfloat16),
             (skew, 100, torch.float32), (skew, 96, torch.float32)]
    for ids, H, dt in cases:
        V = int(ids.max()) + 7
        w = torch.randn(V, H, device="cuda").to(dt).requires_grad_()
        g = torch.randn(ids.numel(), H, device="cuda").to(dt)
        grads = []
        for _ in range(2):
            w.grad = None
            fb.embedding(ids, w).backward(g)
            grads.append(w.grad.clone())
        assert torch.equal(grads[0], grads[1])
        ref = torch.zeros(V, H, device="cuda", dtype=torch.float64).index_add_(0, ids, g.double())
        tol = 1e-2 * max(1.0, float(ref.abs().max()) / 8) if dt == torch.bfloat16 else 1e-4 * float(ref.abs().max())
        torch.testing.assert_close(grads[0].double(), ref, rtol=1e-2, atol=tol)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(1, 768), (7, 3072), (32, 3072), (64, 2304), (65, 768), (4096, 2304)])
def test_col_sum_matches_fp64(M, N):
    """Bias-gradient column sums (csrc/fused_bert.hip: one-pass kernel up to 64 rows, partials + ordered reduce
    above) against fp64, fp32 and bf16 inputs / outputs; run-to-run identical."""
    from mifx.ops import fused_bert as fb

    torch.manual_seed(M)
    for dt, odt in ((torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32)):
        x = torch.randn(M, N, device="cuda").to(dt)
        a, b = fb.col_sum(x, odt), fb.col_sum(x, odt)
        assert torch.equal(a, b) and a.dtype == odt
        ref = x.double().sum(0)
        tol = (2e-2 if odt == torch.bfloat16 else 1e-4) * (1 + float(ref.abs().max()))
        torch.testing.assert_close(a.double(), ref, rtol=2e-2, atol=tol)
