"""BatchNorm + ReLU folded into the consumer 1x1 convolution's GEMM operands (csrc/gemm8.hip AX: gemm8_nt_bnx, grouped
TN BNX problems; mifx.ops.conv1x1.bn_conv1x1): the kernels must equal the stored-activation path exactly (same fused
multiply-add, rounding and accumulation order), and the fused autograd node must match BatchNorm + conv (fp32
PyTorch reference)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _apply(x2, ax):
    """relu(x scale + shift) rounded to bf16 by the BatchNorm apply kernel (csrc/bn_relu.hip)."""
    from mifx.ops import bn_relu
    from mifx.ops._lib import check, ptr, stream_handle

    y = torch.empty_like(x2)
    check(bn_relu._fns()["apply"](1, ptr(x2), x2.shape[0], x2.shape[1], ptr(ax[0]), ptr(ax[1]), 1, ptr(y),
                                  stream_handle(x2.device)), "apply")
    return y


def _ax(k, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    sc = torch.randn(k, device="cuda", generator=g) * 0.5
    sh = torch.randn(k, device="cuda", generator=g) * 0.3
    return torch.stack([sc, sh]).contiguous()


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("epi", [0, 5, 6])
def test_nt_bnx_equals_stored_activation(cfg, epi):
    from mifx.ops import gemm as hg

    bm, bn = hg.gemm8_configs()[cfg]
    M, N, K = 2 * 256, 2 * max(bn, 128), 320
    torch.manual_seed(cfg)
    x = (torch.randn(M, K, device="cuda") * 1.5 + 0.2).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16) if epi == 6 else None
    ax = _ax(K, 7 + cfg)
    act = _apply(x, ax)
    y0, p0 = hg.gemm8_nt(act, w, r, epi, cfg=cfg)
    y1, p1 = hg.gemm8_nt_bnx(x, w, ax, epi, r=r, cfg=cfg)
    assert torch.equal(y0, y1)
    if epi:
        assert torch.equal(p0, p1)
    ref = act.float() @ w.float().t() + (r.float() if r is not None else 0)
    torch.testing.assert_close(y1.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N,T", [(256, 256, 4096), (64, 256, 2048), (256, 64, 2048), (128, 384, 2048)])
def test_grouped_bnx_equals_stored_activation(M, N, T):
    """dW = dY^T relu(X scale + shift) in the grouped split-K launch (128 x 128, narrow-M, narrow-N tiles)
    equals the product with the stored activation, bit for bit, and the fp32 reference."""
    from mifx.ops import gemm as hg

    torch.manual_seed(M + N)
    dy = torch.randn(T, M, device="cuda").to(torch.bfloat16)
    x = (torch.randn(T, N, device="cuda") + 0.1).to(torch.bfloat16)
    ax = _ax(N, 11)
    act = _apply(x, ax)
    c0 = torch.zeros(M, N, device="cuda")
    c1 = torch.zeros(M, N, device="cuda")
    hg.gemm8_tn_grouped([(dy, act, c0)], chunk=1024)
    hg.gemm8_tn_grouped([(dy, x, c1, ax, 1024)])
    assert torch.equal(c0, c1)
    torch.testing.assert_close(c1, dy.float().t() @ act.float(), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("defer,bnx_dw", [(False, False), (True, False), (True, True)])
@pytest.mark.parametrize("res", [False, True])
def test_bn_conv1x1_matches_bn_then_conv(defer, bnx_dw, res, monkeypatch):
    """bn_conv1x1 (activation never stored) vs BatchNormReLU2d + conv in fp32: output, output statistics, running
    statistics and the gradients of x (incl. an alias consumer), gamma, beta, w and the residual."""
    from mifx.ops import conv1x1 as c1
    from mifx.ops import gemm as hg

    monkeypatch.setattr(c1, "BN_FOLD", True)
    monkeypatch.setattr(c1, "_BNX_DW", bnx_dw)  # dW from the grouped operand transform / the re-derived activation
    from mifx.ops.bn_relu import BatchNormReLU2d
    from mifx.ops.conv1x1 import bn_conv1x1, bn_conv_eligible

    torch.manual_seed(3)
    n, c, h, cout = 4, 256, 16, 512
    x0 = (torch.randn(n, c, h, h, device="cuda") * 1.3 + 0.4).to(torch.bfloat16) \
        .contiguous(memory_format=torch.channels_last)
    xm = x0.permute(0, 2, 3, 1).reshape(-1, c).float()
    T = xm.shape[0] // 128  # per-tile (mean, M2) of x, as a producing GEMM would hand them over
    tiles = xm.view(T, 128, c)
    mu = tiles.mean(1)
    part = torch.stack([mu, ((tiles - mu[:, None]) ** 2).sum(1)]).contiguous()
    w = (torch.randn(cout, c, 1, 1, device="cuda") * c ** -0.5).requires_grad_()
    bn = BatchNormReLU2d(c).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    r0 = torch.randn(n, cout, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x = x0.detach().clone().requires_grad_()
    r = r0.detach().clone().requires_grad_() if res else None
    assert bn_conv_eligible(x, part, bn, w)
    g = torch.randn(n, cout, h, h, device="cuda")
    ga = torch.randn(n, c, h, h, device="cuda")
    if defer:
        with hg.deferred_weight_grads():
            out, opart, xa = bn_conv1x1(x, part, bn, w, residual=r)
            (out.float() * g).sum().add((xa.float() * ga).sum()).backward()
        hg.flush_weight_grads()
    else:
        out, opart, xa = bn_conv1x1(x, part, bn, w, residual=r)
        (out.float() * g).sum().add((xa.float() * ga).sum()).backward()
    # fp32 reference
    xr = x0.detach().float().requires_grad_()
    gr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    rm, rv = torch.zeros(c, device="cuda"), torch.ones(c, device="cuda")
    a = F.relu(F.batch_norm(xr, rm, rv, gr, br, True, 0.1, 1e-5))
    rr = r0.float().requires_grad_() if res else None
    o = F.conv2d(a, wr.to(torch.bfloat16).float()) + (rr if res else 0)
    (o * g).sum().add((xr * ga).sum()).backward()
    torch.testing.assert_close(out.float(), o, rtol=3e-2, atol=3e-2 * o.abs().max().item())
    of = out.float().permute(0, 2, 3, 1).reshape(-1, cout).double()
    torch.testing.assert_close(opart[0].double().mean(0), of.mean(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(bn.running_mean, rm, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, rv, rtol=1e-3, atol=1e-4)
    for got, want in ((x.grad.float(), xr.grad), (bn.weight.grad, gr.grad), (bn.bias.grad, br.grad),
                      (w.grad, wr.grad)) + (((r.grad.float(), rr.grad),) if res else ()):
        torch.testing.assert_close(got, want, rtol=5e-2, atol=5e-2 * want.abs().max().item())
