"""Ping-pong pipelined GEMM (csrc/gemm8.hip) against a plain PyTorch fp32 reference of the same op: every tile
configuration (the 64-wide narrow tiles included), every epilogue (none / bias / bias + GELU with the saved pre-bias product / + R / GELU backward with
column sums / BatchNorm statistics), bf16 and fp32 biases, K from one to many K-tiles (the prologue, steady state
and tail of the DMA schedule)."""
import pytest
import torch

from mifx.ops import gemm


def test_gemm8_pick_prefers_full_waves(monkeypatch):
    monkeypatch.setattr(gemm, "gemm8_configs", lambda: ((256, 256), (256, 128), (128, 256), (128, 128)))
    assert gemm.gemm8_pick(4096, 4096, 4096) == 0
    assert gemm.gemm8_pick(4096, 768, 768) in (1, 2, 3)  # 256x256 leaves 48 workgroups on 256 CUs
    assert gemm.gemm8_pick(100, 768, 768) is None
    assert gemm.gemm8_pick(4096, 768, 100) is None


def _operands(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    return x, w


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("K", [64, 128, 192, 640])
def test_gemm8_plain_matches_fp32(cfg, K):
    bm, bn = gemm.gemm8_configs()[cfg]
    M, N = 3 * bm, 2 * bn
    x, w = _operands(M, N, K, cfg * 31 + K)
    y, _ = gemm.gemm8_nt(x, w, cfg=cfg)
    ref = x.float() @ w.float().t()
    # bf16 output: one rounding of the fp32 accumulation
    assert ((y.float() - ref).abs() <= 2 ** -8 * ref.abs() + 1e-3).all()


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("bias_dtype", [torch.bfloat16, torch.float32])
def test_gemm8_epilogues_match_fp32(cfg, bias_dtype):
    bm, bn = gemm.gemm8_configs()[cfg]
    M, N, K = 2 * bm, 3 * bn, 320
    x, w = _operands(M, N, K, 7 + cfg)
    b = (torch.rand(N, device="cuda") - 0.5).to(bias_dtype)
    prod = x.float() @ w.float().t()
    tol = 2e-2 * prod.abs().max().item()
    y, _ = gemm.gemm8_nt(x, w, b, 1, cfg=cfg)
    assert (y.float() - (prod + b.float())).abs().max().item() <= tol
    y, z = gemm.gemm8_nt(x, w, b, 2, cfg=cfg)
    assert (z.float() - prod).abs().max().item() <= tol
    ref = torch.nn.functional.gelu(z.float() + b.float())
    assert (y.float() - ref).abs().max().item() <= 2 ** -7 * ref.abs().max().item()
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    y, _ = gemm.gemm8_nt(x, w, r, 3, cfg=cfg)
    assert (y.float() - (prod + r.float())).abs().max().item() <= tol
    if bn == 64:  # (the narrow tiles carry no GELU-backward epilogue)
        return
    # GELU backward: dZ = (X W^T) o GELU'(Z + b), per-tile column sums of the stored dZ
    zz = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    dz, part = gemm.gemm8_nt(x, w, b, 4, cfg=cfg, z=zz)
    u = (zz.float() + b.float()).requires_grad_()
    gd, = torch.autograd.grad(torch.nn.functional.gelu(u), u, torch.ones_like(u))
    ref = prod * gd
    assert (dz.float() - ref).abs().max().item() <= 2e-2 * ref.abs().max().item()
    assert part.shape == (M // bm, N)
    colref = dz.float().view(M // bm, bm, N).sum(1)
    assert torch.allclose(part, colref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("add", [False, True])
def test_gemm8_stats_epilogue(cfg, add):
    """The BatchNorm-statistics epilogue: per-tile column mean and sum of squared deviations (M2) of the STORED bf16
    output (with add: of the stored Y = X W^T + R); the output itself through the staged 16-byte stores. A large
    column offset checks the two-pass form does not cancel."""
    bm, bn = gemm.gemm8_configs()[cfg]
    M, N, K = 4 * bm, 2 * bn, 256
    x, w = _operands(M, N, K, 100 + cfg)
    r = (torch.randn(M, N, device="cuda") + 40.0).to(torch.bfloat16) if add else None
    y, part = gemm.gemm8_nt(x, w, r, 6 if add else 5, cfg=cfg)
    ref = x.float() @ w.float().t() + (r.float() if add else 0)
    assert ((y.float() - ref).abs() <= 2 ** -8 * ref.abs() + 1e-3).all()
    yf = y.float().view(M // bm, bm, N)
    mean = yf.mean(1)
    m2 = ((yf - mean[:, None, :]) ** 2).sum(1)
    assert part.shape == (2, M // bm, N)
    assert torch.allclose(part[0], mean, rtol=1e-5, atol=1e-4)
    assert torch.allclose(part[1], m2, rtol=1e-3, atol=1e-2)


@pytest.mark.gpu
def test_gemm8_deterministic():
    x, w = _operands(512, 512, 1024, 5)
    a, _ = gemm.gemm8_nt(x, w, cfg=0)
    b, _ = gemm.gemm8_nt(x, w, cfg=0)
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [0, 1])
def test_gemm8_tn_grouped_matches_fp32(cfg):
    """One grouped launch of several TN products C_i = A_i^T B_i (token-major operands, different shapes and token
    counts) against fp32 references; prologue / steady state / tail of the DMA schedule (T from 64 to 1024)."""
    bm = 256 if cfg == 0 else 128
    tile128 = cfg == 1
    g = torch.Generator(device="cuda").manual_seed(11 + cfg)
    shapes = [(bm, bm, 64), (3 * bm, bm, 128), (bm, 2 * bm, 1024), (2 * bm, 3 * bm, 320), (bm, bm, 192)]
    probs, refs = [], []
    for M, N, T in shapes:
        a = (torch.rand(T, M, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        b = (torch.rand(T, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
        c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        probs.append((a, b, c))
        refs.append(a.float().t() @ b.float())
    tiles = gemm.gemm8_tn_grouped(probs, tile128=tile128)
    assert tiles == sum((M // bm) * (N // bm) for M, N, _ in shapes)
    for (_, _, c), ref in zip(probs, refs):
        assert ((c.float() - ref).abs() <= 2 ** -8 * ref.abs() + 1e-2).all()


@pytest.mark.gpu
def test_deferred_weight_grads_equal_reference():
    """hg.linear / hg.ffn inside deferred_weight_grads(): the backward records the weight gradients, one grouped
    flush writes them into .grad; they match the fp32 reference products, input gradients are unchanged."""
    torch.manual_seed(3)
    T, H, F_ = 512, 256, 768
    x = (torch.rand(T, H, device="cuda") * 2 - 1).to(torch.bfloat16).requires_grad_()
    w1 = ((torch.rand(H, H, device="cuda") * 2 - 1) / 16).to(torch.bfloat16).requires_grad_()
    wi = ((torch.rand(F_, H, device="cuda") * 2 - 1) / 16).to(torch.bfloat16).requires_grad_()
    bi = torch.zeros(F_, device="cuda", dtype=torch.bfloat16).requires_grad_()
    wo = ((torch.rand(H, F_, device="cuda") * 2 - 1) / 16).to(torch.bfloat16).requires_grad_()

    def run(defer):
        for t in (x, w1, wi, bi, wo):
            t.grad = None
        h = gemm.linear(x, w1, force=True)
        y = gemm.ffn(h, wi, bi, wo)
        gy = torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y).to(y.dtype)
        if defer:
            with gemm.deferred_weight_grads():
                y.backward(gy)
            assert gemm.flush_weight_grads() == 3
        else:
            y.backward(gy)
        return [t.grad.clone() for t in (x, w1, wi, wo)]

    ref = run(False)
    got = run(True)
    assert torch.equal(got[0], ref[0])  # the input gradient does not depend on the deferral
    for g_, r_ in zip(got[1:], ref[1:]):
        err = ((g_.float() - r_.float()).abs().max() / r_.float().abs().max()).item()
        assert err < 1e-2, err


@pytest.mark.gpu
def test_gemm8_tn_grouped_quarter_tile_tail():
    """260 full-size tiles: the 4 beyond the last whole wave of 256 run as 16 quarter-size tiles (the tail path)."""
    g = torch.Generator(device="cuda").manual_seed(5)
    M, N, T = 256 * 20, 256 * 13, 128
    a = (torch.rand(T, M, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    b = (torch.rand(T, N, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    assert gemm.gemm8_tn_grouped([(a, b, c)]) == 260
    ref = a.float().t() @ b.float()
    assert ((c.float() - ref).abs() <= 2 ** -8 * ref.abs() + 1e-2).all()


@pytest.mark.gpu
def test_gemm8_tn_grouped_fp32_split_accumulates():
    """fp32 destinations: C += A^T B with the token range split into chunks (the last one short), mixed 256 / 128
    tiles, bf16 and fp32 problems in one launch."""
    g = torch.Generator(device="cuda").manual_seed(9)
    shapes = [(128, 512, 12544, True), (512, 256, 4096 + 640, True), (256, 256, 1024, False)]
    probs, refs = [], []
    for M, N, T, f32 in shapes:
        a = (torch.rand(T, M, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
        b = (torch.rand(T, N, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
        c0 = torch.randn(M, N, device="cuda") if f32 else None
        c = c0.clone() if f32 else torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        probs.append((a, b, c))
        refs.append(a.float().t() @ b.float() + (c0 if f32 else 0))
    items = gemm.gemm8_tn_grouped(probs, chunk=2048)
    # 4 tiles of 128 x 128 x 7 chunks (the last 256 rows) + 2 tiles of 256 x 256 x 3 chunks + 1 bf16 tile
    assert items == 4 * 7 + 2 * 3 + 1
    for (_, _, c), ref in zip(probs, refs):
        err = ((c.float() - ref).abs().max() / ref.abs().max()).item()
        assert err < (1e-5 if c.dtype == torch.float32 else 1e-2), err


@pytest.mark.gpu
@pytest.mark.parametrize("M,N", [(256, 64), (512, 192), (64, 256), (192, 512)])
def test_gemm8_tn_grouped_narrow_fp32(M, N):
    """fp32 split-K weight gradients with a 64-wide dimension on the narrow 256 x 64 / 64 x 256 tiles (duplicated
    DMAs, 64-byte rotated token rows), accumulating into an existing gradient, against fp32."""
    g = torch.Generator(device="cuda").manual_seed(M + N)
    T = 4096 + 640
    a = (torch.rand(T, M, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
    b = (torch.rand(T, N, device="cuda", generator=g) - 0.5).to(torch.bfloat16)
    c = torch.randn(M, N, device="cuda", generator=g)
    want = c + a.float().t() @ b.float()
    gemm.gemm8_tn_grouped([(a, b, c)], chunk=2048)
    torch.testing.assert_close(c, want, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_forward_route_to_gemm8_matches_fp32(monkeypatch):
    """G8_FWD (MIFX_G8_FWD): the BERT forward projections routed to the 8-wave kernel -- linear with bias, the fused
    FFN (bias + GELU epilogue with its Z output, then FFN-out) -- against fp32 references, forward and backward."""
    from mifx.ops import native_stats  # noqa: F401  (dispatch counters are exercised on the way)

    dev = torch.device("cuda")
    M, H, I = 512, 256, 512
    monkeypatch.setattr(gemm, "G8_FWD", {(M, 3 * H, H): 0, (M, I, H): 3, (M, H, I): 5})
    g = torch.Generator(device=dev).manual_seed(3)
    x = (torch.randn(M, H, device=dev, generator=g) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(3 * H, H, device=dev, generator=g) * 0.05).bfloat16().requires_grad_()
    b = (torch.randn(3 * H, device=dev, generator=g) * 0.1).bfloat16().requires_grad_()
    y = gemm.linear(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    assert (y.float() - ref).norm() / ref.norm() < 1e-2
    w1 = (torch.randn(I, H, device=dev, generator=g) * 0.05).bfloat16().requires_grad_()
    b1 = (torch.randn(I, device=dev, generator=g) * 0.1).bfloat16().requires_grad_()
    w2 = (torch.randn(H, I, device=dev, generator=g) * 0.05).bfloat16().requires_grad_()
    o = gemm.ffn(x, w1, b1, w2)
    xf = x.detach().float().requires_grad_()
    w1f, b1f, w2f = (t.detach().float().requires_grad_() for t in (w1, b1, w2))
    of = torch.nn.functional.gelu(xf @ w1f.t() + b1f) @ w2f.t()
    assert (o.float() - of).norm() / of.norm() < 2e-2
    go = torch.randn_like(of)
    o.backward(go.bfloat16())
    of.backward(go)
    for a, r in ((w1.grad, w1f.grad), (b1.grad, b1f.grad), (w2.grad, w2f.grad)):
        assert (a.float() - r).norm() / r.norm() < 3e-2


@pytest.mark.gpu
def test_dx_route_to_gemm8_matches_fp32(monkeypatch):
    """G8_DX (MIFX_G8_DX): the projections' input gradient dY W on the 8-wave kernel against the transposed weight,
    with and without the residual gradient folded in as the C operand (GradSlot), vs fp32."""
    dev = torch.device("cuda")
    M, K, N = 512, 768, 256  # dX [M, N] = dY [M, K] . W [K, N]
    monkeypatch.setattr(gemm, "G8_DX", {(M, N, K): 5})
    g = torch.Generator(device=dev).manual_seed(5)
    x = (torch.randn(M, N, device=dev, generator=g) * 0.5).bfloat16().requires_grad_()
    w = (torch.randn(K, N, device=dev, generator=g) * 0.05).bfloat16().requires_grad_()
    dy = torch.randn(M, K, device=dev, generator=g).bfloat16()
    gemm.linear(x, w, force=True).backward(dy)  # (force: the _Linear node, whose backward is _dx)
    ref = dy.float() @ w.detach().float()
    assert (x.grad.float() - ref).norm() / ref.norm() < 1e-2
    r = torch.randn(M, N, device=dev, generator=g).bfloat16()
    slot = gemm.GradSlot()
    slot.g = r
    out = gemm._dx(dy, w.detach(), slot)
    ref2 = ref + r.float()
    assert (out.float() - ref2).norm() / ref2.norm() < 1e-2
