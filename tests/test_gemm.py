"""Hand-written MFMA GEMM (csrc/gemm.hip) against a plain PyTorch fp32 reference of the same op: every tile
configuration, every epilogue (none / bias / bias + GELU with the saved pre-bias product), bf16 and fp32 biases,
and the autograd wrappers' gradients."""
import pytest
import torch

from mifx.ops import gemm


def _ref(x, w, b=None, gelu=False):
    z = x.float() @ w.float().t()
    y = z + b.float() if b is not None else z
    return torch.nn.functional.gelu(y) if gelu else y, z


def test_pick_config_prefers_full_waves(monkeypatch):
    monkeypatch.setattr(gemm, "configs", lambda: ((256, 256), (256, 128), (128, 128), (128, 256)))
    gemm.TUNED.clear()
    assert gemm.pick_config(4096, 3072, 768) is not None
    assert gemm.pick_config(4096, 768, 768) in (1, 2, 3)  # 256x256 leaves 48 workgroups on 256 CUs
    assert gemm.pick_config(100, 768, 768) is None  # no configuration tiles M = 100
    assert gemm.pick_config(4096, 768, 100) is None  # K % 64


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", list(range(19)))
@pytest.mark.parametrize("epi,bias_dtype", [(0, None), (1, torch.bfloat16), (1, torch.float32), (2, torch.bfloat16),
                                            (2, torch.float32)])
def test_gemm_nt_matches_fp32_reference(cfg, epi, bias_dtype):
    torch.manual_seed(cfg * 7 + epi)
    bm, bn = gemm.configs()[cfg]
    M, N, K = 2 * bm, 3 * bn, 320
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    b = (torch.rand(N, device="cuda") - 0.5).to(bias_dtype) if bias_dtype is not None else None
    y, z = gemm.gemm_nt(x, w, b, epi, cfg=cfg)
    ref, zref = _ref(x, w, b, gelu=epi == 2)
    tol = 2e-2 * ref.abs().max().item()
    assert (y.float() - ref).abs().max().item() <= tol
    if epi == 2:
        assert (z.float() - zref).abs().max().item() <= 2e-2 * zref.abs().max().item()
        # the epilogue == the unfused bias_gelu kernel applied to the stored product z, up to one bf16 rounding step
        # (branch-free erf, |error| <= 1.5e-7, against the library erff)
        from mifx.ops import fused_bert as fb

        ref_y = fb.bias_gelu(z, b).float()
        assert (y.float() - ref_y).abs().max().item() <= 2 ** -8 * ref_y.abs().max().item()
        assert (y != fb.bias_gelu(z, b)).float().mean().item() < 0.01


@pytest.mark.gpu
def test_linear_bias_gelu_autograd_matches_reference():
    torch.manual_seed(1)
    M, K, N = 512, 256, 768
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16).requires_grad_()
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16).requires_grad_()
    b = (torch.rand(N, device="cuda") - 0.5).to(torch.bfloat16).requires_grad_()
    assert gemm.eligible(x, w)
    y = gemm.linear_bias_gelu(x, w, b, force=True)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.gelu(xr @ wr.t() + br)
    yr.backward(g.float())
    assert (y.float() - yr).abs().max().item() <= 2e-2 * yr.abs().max().item()
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (got.float() - ref).abs().max().item() <= 3e-2 * ref.abs().max().item()


@pytest.mark.gpu
def test_linear_autograd_and_fallback():
    torch.manual_seed(2)
    x = (torch.rand(4, 64, 128, device="cuda") * 2 - 1).to(torch.bfloat16).requires_grad_()
    w = ((torch.rand(256, 128, device="cuda") * 2 - 1) * 0.1).to(torch.bfloat16).requires_grad_()
    b = (torch.rand(256, device="cuda") - 0.5).to(torch.bfloat16).requires_grad_()
    assert gemm.eligible(x, w)
    y = gemm.linear(x, w, b, force=True)
    y.sum().backward()
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.sum().backward()
    assert (y.float() - yr).abs().max().item() <= 2e-2 * yr.abs().max().item()
    for got, ref in ((x.grad, xr.grad), (w.grad, wr.grad), (b.grad, br.grad)):
        assert (got.float() - ref).abs().max().item() <= 3e-2 * ref.abs().max().item()
    # a shape no configuration tiles: F.linear
    x2 = torch.randn(100, 128, device="cuda", dtype=torch.bfloat16)
    assert not gemm.eligible(x2, w.detach())
    assert gemm.linear(x2, w.detach(), b.detach(), force=True).shape == (100, 256)
    # not measured faster for this shape: the library path unless forced
    assert not gemm.preferred(x.detach(), w.detach())


@pytest.mark.gpu
def test_bert_layer_on_hip_gemm_matches_library_path():
    """A small BERT (hidden 256, FFN 1024, 256 tokens: every projection tiles) with hip_gemm on vs off: same
    logits and gradients within bf16 tolerance; the HIP path must really run (eligible shapes)."""
    from mifx.models.bert import BertConfig, BertForSequenceClassification

    import os

    os.environ["MIFX_HIP_GEMM"] = "all"  # every tiled projection on the kernel (not only the TUNED shapes)
    out = []
    for hip in (True, False):
        cfg = BertConfig(vocab_size=1000, hidden=256, layers=2, heads=4, intermediate=1024, max_position=64,
                         dropout=0.0, hip_gemm=hip)
        m = BertForSequenceClassification(cfg, seed=0).cuda().to(torch.bfloat16)
        g = torch.Generator().manual_seed(0)
        ids = torch.randint(0, 1000, (4, 64), generator=g).cuda()
        am = torch.ones(4, 64, device="cuda")
        x = torch.zeros(256, 256, device="cuda", dtype=torch.bfloat16)
        assert gemm.eligible(x, m.layers[0].ffn_in.weight) and gemm.eligible(x, m.layers[0].qkv.weight)
        logits = m(ids, None, am)
        logits.float().sum().backward()
        out.append((logits.float().detach(), m.layers[0].ffn_in.weight.grad.float(), m.layers[0].qkv.weight.grad.float()))
    del os.environ["MIFX_HIP_GEMM"]
    for a, b in zip(out[0], out[1]):
        assert (a - b).abs().max().item() <= 5e-2 * b.abs().max().item() + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1000, 1000, 1000), (1, 7, 3), (65, 129, 17), (300, 64, 1000), (64, 64, 64)])
def test_matmul_f32_edge_tiles_match_fp64(M, N, K):
    """csrc/gemm_f32.hip: exact fp32 MFMA products / sums with ragged edges (zero-filled tile loads, masked
    stores), against an fp64 reference: the KN18 anchor (1000 x 1000) and shapes that are no tile multiple."""
    from mifx.ops.gemm import matmul_f32

    g = torch.Generator().manual_seed(M * 7 + N + K)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(K, N, generator=g)
    c = matmul_f32(a.cuda(), b.cuda()).cpu()
    ref = (a.double() @ b.double())
    err = (c.double() - ref).abs().max().item()
    # fp32 accumulation over K terms of O(1) products: a few ulps of sqrt(K)-sized sums
    assert err <= 4e-6 * max(1.0, K ** 0.5) * ref.abs().max().item(), err


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", list(range(7)))
@pytest.mark.parametrize("with_r", [False, True])
def test_gemm_nn_matches_fp32_reference(cfg, with_r):
    """csrc/gemm_nn.hip (dX = dY W [+ R]) against the fp32 product: every configuration, with and without the
    folded C operand, on a shape of several tiles in both dimensions and 5 K-tiles (ring wrap-around)."""
    torch.manual_seed(100 + cfg)
    bm, bn, _ = gemm.nn_configs()[cfg]
    M, N, K = 2 * bm, 3 * bn, 320
    a = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    b = ((torch.rand(K, N, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    r = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16) if with_r else None
    c = gemm.gemm_nn(a, b, r, cfg=cfg)
    ref = a.float() @ b.float() + (r.float() if with_r else 0)
    assert (c.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.gpu
def test_dx_routes_to_nn_kernel_and_matches_library(monkeypatch):
    """_Linear's input gradient on the NN kernel (forced via NN_TUNED) equals the library's, including the
    GradSlot residual fold; the native counter records the kernel."""
    from mifx.ops import native_stats

    torch.manual_seed(5)
    M, K, N = 512, 384, 192  # x [M, K] -> y [M, N]; dX = dY[M, N] W[N, K]
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16).requires_grad_()
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    ref = torch.autograd.grad(torch.nn.functional.linear(x, w), x, dy)[0]
    monkeypatch.setitem(gemm.NN_TUNED, (M, K, N), gemm.nn_pick(M, K, N))
    native_stats.reset()
    got = torch.autograd.grad(gemm.linear(x, w, force=True), x, dy)[0]
    assert native_stats.snapshot()["gemm_dX"]["native"] == 1
    torch.testing.assert_close(got.float(), ref.float(), rtol=2e-2, atol=2e-2)
    slot = gemm.GradSlot()
    res = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    slot.g = res
    got2 = torch.autograd.grad(gemm.linear(x, w, force=True, slot=slot), x, dy)[0]
    torch.testing.assert_close(got2.float(), (ref.float() + res.float()), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
def test_transpose_and_add_r_epilogue():
    """transpose_bf16 is exact; the NT kernel's R epilogue (epi 3) adds R before the single rounding."""
    torch.manual_seed(9)
    w = torch.randn(192, 320, device="cuda").to(torch.bfloat16)
    assert torch.equal(gemm.transpose(w), w.t().contiguous())
    M, N, K = 256, 192, 384
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    wt = ((torch.rand(N, K, device="cuda") * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    r = (torch.rand(M, N, device="cuda") - 0.5).to(torch.bfloat16)
    y, _ = gemm.gemm_nt(x, wt, r, 3, cfg=12)
    ref = x.float() @ wt.float().t() + r.float()
    assert (y.float() - ref).abs().max().item() <= 1e-2 * ref.abs().max().item()


@pytest.mark.gpu
def test_dx_on_transposed_nt_matches_library(monkeypatch):
    """_Linear's input gradient through the transposed-weight NT path (DX_NT_TUNED) equals the library's, with and
    without the GradSlot residual fold."""
    from mifx.ops import native_stats

    torch.manual_seed(6)
    M, K, N = 512, 384, 192
    x = (torch.randn(M, K, device="cuda") * 0.5).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16).requires_grad_()
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    ref = torch.autograd.grad(torch.nn.functional.linear(x, w), x, dy)[0]
    monkeypatch.setitem(gemm.DX_NT_TUNED, (M, K, N), 12)
    native_stats.reset()
    got = torch.autograd.grad(gemm.linear(x, w, force=True), x, dy)[0]
    assert native_stats.snapshot()["gemm_dX"]["native"] == 1
    torch.testing.assert_close(got.float(), ref.float(), rtol=2e-2, atol=2e-2)
    slot = gemm.GradSlot()
    res = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    slot.g = res
    got2 = torch.autograd.grad(gemm.linear(x, w, force=True, slot=slot), x, dy)[0]
    torch.testing.assert_close(got2.float(), ref.float() + res.float(), rtol=2e-2, atol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [True, False])
def test_ffn_block_matches_fp32_reference(monkeypatch, fused):
    """gemm.ffn (one autograd node: FFN-in + bias + GELU + FFN-out) against the fp32 composition: forward, the input
    gradient (with a GradSlot residual), both weight gradients and the bias gradient; fused = the dH GEMM with the
    GELU-backward epilogue and in-kernel bias-gradient partials, else dH then the bias_gelu backward kernel."""
    from mifx.ops import native_stats

    torch.manual_seed(11)
    M, H, I = 512, 192, 384
    if fused:
        monkeypatch.setitem(gemm.GELU_BWD_TUNED, (M, I, H), 9)
    else:
        monkeypatch.setenv("MIFX_HIP_GELU_BWD", "0")
    x = (torch.randn(M, H, device="cuda") * 0.7).to(torch.bfloat16).requires_grad_()
    w1 = (torch.randn(I, H, device="cuda") * H ** -0.5).to(torch.bfloat16).requires_grad_()
    b1 = (torch.randn(I, device="cuda") * 0.1).to(torch.bfloat16).requires_grad_()
    w2 = (torch.randn(H, I, device="cuda") * I ** -0.5).to(torch.bfloat16).requires_grad_()
    res = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    slot = gemm.GradSlot()
    native_stats.reset()
    out = gemm.ffn(x, w1, b1, w2, slot=slot)
    g = torch.randn_like(out)
    slot.g = res
    out.backward(g)
    assert native_stats.snapshot()["gemm_dX_gelu_bwd"] == {"native": int(fused), "fallback": int(not fused)}
    xr, w1r, b1r, w2r = (t.detach().float().requires_grad_() for t in (x, w1, b1, w2))
    ref = torch.nn.functional.gelu(xr @ w1r.t() + b1r) @ w2r.t()
    ref.backward(g.float())
    torch.testing.assert_close(out.float(), ref, rtol=3e-2, atol=3e-2)
    for got, want, name in ((x.grad.float(), xr.grad + res.float(), "dx"), (w1.grad.float(), w1r.grad, "dw1"),
                            (b1.grad.float(), b1r.grad, "db1"), (w2.grad.float(), w2r.grad, "dw2")):
        err = (got - want).norm() / want.norm()
        assert err < 2e-2, f"{name}: relative error {err:.4f}"


@pytest.mark.gpu
def test_transpose_cache_batch_refresh():
    """TransposeCache: every registered weight transposed in one launch; refresh() after an in-place update; used by
    _dx only inside use_transposes()."""
    torch.manual_seed(12)
    ws = [torch.randn(r, c, device="cuda").to(torch.bfloat16) for r, c in ((192, 320), (64, 64), (768, 128))]
    tc = gemm.TransposeCache(ws)
    tc.refresh()
    for w in ws:
        assert torch.equal(tc.get(w), w.t().contiguous())
    ws[0].mul_(2)
    assert not torch.equal(tc.get(ws[0]), ws[0].t().contiguous())  # stale until refreshed
    tc.refresh()
    assert torch.equal(tc.get(ws[0]), ws[0].t().contiguous())
    assert gemm.transposed(ws[1]) is not tc.get(ws[1])  # inactive: a fresh transpose
    with gemm.use_transposes(tc):
        assert gemm.transposed(ws[1]) is tc.get(ws[1])
