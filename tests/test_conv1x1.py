"""1x1 convolutions on the pipelined GEMM with BatchNorm statistics / residual add in the epilogue
(mifx.ops.conv1x1, csrc/gemm8.hip), the BatchNorm that consumes those statistics (bn_relu forward_tiles), the deferred
fp32 weight gradients, and the ResNet-50 v2 blocks built on them -- all against plain PyTorch fp32 references."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _x(n, c, h, w, seed, scale=1.0, shift=0.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = (torch.randn(n, c, h, w, device="cuda", generator=g) * scale + shift).to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("cin,cout,res", [(64, 256, False), (256, 128, True), (512, 512, True)])
def test_conv1x1_forward_stats_backward(cin, cout, res):
    from mifx.ops import gemm as hg
    from mifx.ops.conv1x1 import conv1x1, eligible

    x = _x(4, cin, 16, 8, 1).requires_grad_()
    w = (torch.randn(cout, cin, 1, 1, device="cuda") * cin ** -0.5).requires_grad_()
    r = _x(4, cout, 16, 8, 2, 2.0, 5.0).requires_grad_() if res else None
    assert eligible(x, w)
    y, part = conv1x1(x, w, r, stats=True)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.bfloat16
    ref = F.conv2d(x.float(), w.float()) + (r.float() if res else 0)
    assert ((y.float() - ref).abs() <= 2 ** -7 * ref.abs() + 2e-2).all()
    # per-tile statistics of the stored output, combined: the batch mean / variance of y
    M = 4 * 16 * 8
    T = part.shape[1]
    yf = y.float().permute(0, 2, 3, 1).reshape(M, cout)
    tm, tm2 = part[0].double(), part[1].double()
    mean = tm.mean(0)
    var = (tm2.sum(0) + (M // T) * ((tm - mean) ** 2).sum(0)) / M
    torch.testing.assert_close(mean, yf.double().mean(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(var, yf.double().var(0, unbiased=False), rtol=1e-4, atol=1e-5)
    # backward: dX = dY W, dW = dY^T X (hipBLASLt and the deferred grouped TN flush), dR = dY
    gy = _x(4, cout, 16, 8, 3)
    y.backward(gy)
    xr, wr = x.detach().float().requires_grad_(), w.detach().clone().requires_grad_()
    F.conv2d(xr, wr.to(torch.bfloat16).float()).backward(gy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())
    if res:
        assert torch.equal(r.grad, gy)
    w2 = w.detach().clone().requires_grad_()
    y2, _ = conv1x1(x.detach(), w2, r.detach() if res else None, stats=True)
    with hg.deferred_weight_grads():
        y2.backward(gy)
    # (Cin = 64 with Cout % 256: the narrow 256 x 64 grouped tiles)
    assert hg.flush_weight_grads() == (1 if cin % 128 == 0 or cout % 256 == 0 else 0)
    torch.testing.assert_close(w2.grad, wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())


def test_bn_forward_tiles_matches_batchnorm():
    """BatchNormReLU2d.forward_tiles (statistics from the GEMM epilogue) == the module's own forward (statistics
    pass): outputs, running statistics, and the backward through the fused dres path."""
    from mifx.ops.bn_relu import BatchNormReLU2d
    from mifx.ops.conv1x1 import conv1x1

    torch.manual_seed(0)
    x = _x(8, 256, 16, 16, 4)
    w = torch.randn(512, 256, 1, 1, device="cuda") * 256 ** -0.5
    y, part = conv1x1(x, w, stats=True)
    y = y.detach().requires_grad_()
    bn_a, bn_b = BatchNormReLU2d(512).cuda(), BatchNormReLU2d(512).cuda()
    bn_b.load_state_dict(bn_a.state_dict())
    out_a, alias = bn_a.forward_tiles(y, part)
    y2 = y.detach().clone().requires_grad_()
    out_b = bn_b(y2)
    torch.testing.assert_close(out_a.float(), out_b.float(), rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(bn_a.running_mean, bn_b.running_mean, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(bn_a.running_var, bn_b.running_var, rtol=1e-4, atol=1e-5)
    g = _x(8, 512, 16, 16, 5)
    gp = _x(8, 512, 16, 16, 6)
    torch.autograd.backward([out_a, alias], [g, gp])
    out_b.backward(g)
    torch.testing.assert_close(y.grad.float(), (y2.grad + gp).float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(bn_a.weight.grad, bn_b.weight.grad, rtol=1e-3, atol=1e-3)


def test_resnet_fused_1x1_matches_unfused_path():
    """ResNet-50 v2 blocks (bf16 autocast, channels_last) with the fused 1x1 path vs the routed MIOpen path, both
    against the fp32 network: logits, every parameter gradient (with and without the deferred grouped weight
    gradients) and the running statistics. The bf16 paths differ from fp32 by bf16 rounding amplified through the
    train-mode BatchNorms; the fused path must be as close to fp32 as the unfused one."""
    import mifx.models.resnet as R
    from mifx.ops import gemm as hg

    torch.manual_seed(0)
    base = R.ResNetV2((2, 2, 1, 1), 10).cuda().to(memory_format=torch.channels_last)
    x = torch.rand(8, 3, 128, 128, device="cuda").contiguous(memory_format=torch.channels_last)
    gout = torch.randn(8, 10, device="cuda")

    def run(fused, defer, amp=True):
        m = copy.deepcopy(base)
        saved = R.FUSED_1X1
        R.FUSED_1X1 = fused
        try:
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
                out = m(x).float()
            if defer:
                with hg.deferred_weight_grads():
                    out.backward(gout)
                assert hg.flush_weight_grads() > 0
            else:
                out.backward(gout)
        finally:
            R.FUSED_1X1 = saved
        return m, out

    saved = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        mr, orf = run(False, False, amp=False)  # fp32 reference (the fused path needs bf16: not taken)
    finally:
        torch.backends.cudnn.allow_tf32 = saved
    m0, o0 = run(False, False)
    m1, o1 = run(True, False)
    m2, o2 = run(True, True)
    from mifx.ops import conv1x1 as c1

    saved_fold = c1.BN_FOLD
    c1.BN_FOLD = not saved_fold  # the other BatchNorm mode: folded into the consumer GEMMs / applied by own pass
    try:
        m3, o3 = run(True, True)
    finally:
        c1.BN_FOLD = saved_fold
    e0 = (o0 - orf).abs().max().item()
    assert (o1 - orf).abs().max().item() <= 2 * e0 + 1e-2
    assert (o2 - orf).abs().max().item() <= 2 * e0 + 1e-2
    assert (o3 - orf).abs().max().item() <= 2 * e0 + 1e-2
    pr, p0, p1, p2, p3 = (dict(m.named_parameters()) for m in (mr, m0, m1, m2, m3))

    def rel(a, b):
        return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()

    rows = []
    for n in pr:
        r0, r1, r2 = rel(p0[n].grad, pr[n].grad), rel(p1[n].grad, pr[n].grad), rel(p2[n].grad, pr[n].grad)
        r3 = rel(p3[n].grad, pr[n].grad)
        rows.append(f"{n}: unfused {r0:.3e} fused {r1:.3e} fused+deferred {r2:.3e} other BN mode {r3:.3e}")
        assert r1 <= 2 * r0 + 2e-2 and r2 <= 2 * r0 + 2e-2 and r3 <= 2 * r0 + 2e-2, "\n".join(rows)
    b0, b1, br = dict(m0.named_buffers()), dict(m1.named_buffers()), dict(mr.named_buffers())
    for n in b0:
        if n.endswith(("running_mean", "running_var")):
            torch.testing.assert_close(b1[n], br[n], rtol=3e-2, atol=3e-3)


def test_gemm8_bnbwd_epilogue_partials():
    """EPI_BNBWD: the stored dY plus per-tile (sum g, sum g xhat) of the BatchNorm + ReLU backward, against fp32
    sums of the same stored values."""
    from mifx.ops import gemm as hg

    g = torch.Generator(device="cuda").manual_seed(7)
    M, N, K = 1024, 256, 512
    a = (torch.randn(M, K, device="cuda", generator=g)).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    xb = (torch.randn(M, N, device="cuda", generator=g) * 2 + 0.5).to(torch.bfloat16)
    mean = torch.randn(N, device="cuda", generator=g) * 0.3
    rstd = torch.rand(N, device="cuda", generator=g) + 0.5
    gamma = torch.randn(N, device="cuda", generator=g)
    beta = torch.randn(N, device="cuda", generator=g) * 0.2
    stats = torch.stack([mean, rstd, gamma * rstd, beta - mean * gamma * rstd]).contiguous()
    for cfg, (bm, bn) in enumerate(hg.gemm8_configs()):
        y, part = hg.gemm8_nt(a, w, xb, 8, cfg=cfg, z=stats)
        ref = a.float() @ w.float().t()
        assert ((y.float() - ref).abs() <= 2 ** -7 * ref.abs() + 1e-2).all()
        xf = xb.float()
        mask = (xf * stats[2] + stats[3]) > 0
        gg = torch.where(mask, y.float(), torch.zeros_like(ref))
        xhat = (xf - mean) * rstd
        T = M // bm
        assert part.shape == (2, T, N)
        torch.testing.assert_close(part[0], gg.view(T, bm, N).sum(1), rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(part[1], (gg * xhat).view(T, bm, N).sum(1), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("second_consumer", [False, True])
def test_conv1x1_bn_coupled_backward(second_consumer):
    """A BatchNorm + ReLU whose output feeds a 1x1 conv with bn_input=True takes its backward sums from the dX GEMM's
    epilogue: gradients equal the uncoupled path's; when a second consumer's gradient is accumulated into the same
    buffer (autograd's in-place accumulation) the node must notice and reduce itself."""
    from mifx.ops.bn_relu import BatchNormReLU2d
    from mifx.ops.conv1x1 import conv1x1

    torch.manual_seed(1)
    x0 = _x(4, 256, 16, 16, 11, 1.5, 0.3)
    w = torch.randn(512, 256, 1, 1, device="cuda") * 256 ** -0.5
    gy = _x(4, 512, 16, 16, 12)
    bn_ref = BatchNormReLU2d(256).cuda()
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.2, 0.2)
    grads = []
    for couple in (False, True):
        bn = copy.deepcopy(bn_ref)
        x = x0.detach().clone().requires_grad_()
        wc = w.detach().clone().requires_grad_()
        pre = bn(x)
        y, _ = conv1x1(pre, wc, bn_input=couple)
        loss = (y.float() * gy.float()).sum()
        if second_consumer:
            loss = loss + (pre.float() * 0.25).sum()
        loss.backward()
        grads.append((x.grad.float(), bn.weight.grad, bn.bias.grad, wc.grad))
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * b.abs().max().item())
    # and against fp32
    xr = x0.detach().float().requires_grad_()
    wr = bn_ref.weight.detach().clone().requires_grad_()
    br = bn_ref.bias.detach().clone().requires_grad_()
    pre = F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5))
    loss = (F.conv2d(pre, w) * gy.float()).sum()
    if second_consumer:
        loss = loss + (pre * 0.25).sum()
    loss.backward()
    for a, b in zip(grads[1][:3], (xr.grad, wr.grad, br.grad)):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * b.abs().max().item())


@pytest.mark.parametrize("couple", [False, True])
@pytest.mark.parametrize("stride,cin,cs,c1", [(2, 256, 512, 128), (1, 64, 256, 64)])
def test_proj_pair_matches_separate_convs(couple, stride, cin, cs, c1):
    """1x1 projection shortcut (strided, or stride 1 as in ResNet-50's stage 1) + 1x1 conv1 as one node
    (mifx.ops.conv1x1.proj_pair): outputs, BN1 statistics, and the summed input gradient written by conv1's dX GEMM
    (EPI_ADD_BNBWD, with the upstream BatchNorm's sums when coupled) against fp32 PyTorch."""
    from mifx.ops.bn_relu import BatchNormReLU2d
    from mifx.ops.conv1x1 import proj_pair, proj_pair_eligible

    torch.manual_seed(2)
    x0 = _x(4, cin, 16, 16, 21, 1.2, 0.2)
    wsc = (torch.randn(cs, cin, 1, 1, device="cuda") * cin ** -0.5).contiguous(memory_format=torch.channels_last)
    w1 = (torch.randn(c1, cin, 1, 1, device="cuda") * cin ** -0.5).contiguous(memory_format=torch.channels_last)
    gsc = _x(4, cs, 16 // stride, 16 // stride, 22)
    g1 = _x(4, c1, 16, 16, 23)
    bn = BatchNormReLU2d(cin).cuda()
    x = x0.detach().clone().requires_grad_()
    a, b = wsc.detach().clone().requires_grad_(), w1.detach().clone().requires_grad_()
    pre = bn(x)
    assert proj_pair_eligible(pre, a, stride, b)
    sc, y1, part = proj_pair(pre, a, stride, b, bn_input=couple)
    (sc.float() * gsc.float()).sum().add((y1.float() * g1.float()).sum()).backward()
    # fp32 reference
    xr = x0.detach().float().requires_grad_()
    wr, br = bn.weight.detach().clone().requires_grad_(), bn.bias.detach().clone().requires_grad_()
    ar, b1r = wsc.detach().clone().requires_grad_(), w1.detach().clone().requires_grad_()
    pr = F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5))
    scr = F.conv2d(pr, ar.to(torch.bfloat16).float(), stride=stride)
    y1r = F.conv2d(pr, b1r.to(torch.bfloat16).float())
    (scr * gsc.float()).sum().add((y1r * g1.float()).sum()).backward()
    torch.testing.assert_close(sc.float(), scr, rtol=3e-2, atol=3e-2)
    torch.testing.assert_close(y1.float(), y1r, rtol=3e-2, atol=3e-2)
    M, T = 4 * 16 * 16, part.shape[1]
    yf = y1.float().permute(0, 2, 3, 1).reshape(M, c1).double()
    torch.testing.assert_close(part[0].double().mean(0), yf.mean(0), rtol=1e-5, atol=1e-5)
    for got, want in ((x.grad.float(), xr.grad), (bn.weight.grad, wr.grad), (bn.bias.grad, br.grad),
                      (a.grad, ar.grad), (b.grad, b1r.grad)):
        torch.testing.assert_close(got, want, rtol=5e-2, atol=5e-2 * want.abs().max().item())


@pytest.mark.parametrize("nb,h,cin,cout", [(4, 16, 256, 512), (2, 15, 128, 256), (8, 16, 512, 1024)])
def test_strided_1x1_center_tap(nb, h, cin, cout):
    """Strided 1x1 convolution as the center tap of the implicit 3x3 GEMM (csrc/gemm8.hip, tap0 = 4): output and
    per-tile BatchNorm statistics against an fp32 conv2d(stride 2), odd input sizes included."""
    from mifx.ops import gemm as hg

    torch.manual_seed(5)
    x = torch.randn(nb, h, h, cin, device="cuda").to(torch.bfloat16)
    w = (torch.randn(cout, cin, device="cuda") * cin ** -0.5).to(torch.bfloat16)
    y, part = hg.gemm8_conv1x1_strided(x, w, 2, epi=5)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float()[:, :, None, None], stride=2)
    ref2 = ref.permute(0, 2, 3, 1).reshape(-1, cout)
    torch.testing.assert_close(y.float(), ref2, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(part[0].double().mean(0), y.float().double().mean(0), rtol=1e-5, atol=1e-5)


def test_proj_pair_deferred_shortcut_weight_grad():
    """Inside deferred_weight_grads(): the shortcut's weight gradient is recorded with the center-tap geometry and
    computed by the grouped TN flush -- equal to the fp32 reference (and the node's other gradients unchanged)."""
    from mifx.ops import gemm as hg
    from mifx.ops.conv1x1 import proj_pair

    torch.manual_seed(6)
    x = _x(4, 256, 16, 16, 31).requires_grad_()
    wsc = (torch.randn(512, 256, 1, 1, device="cuda") * 256 ** -0.5).requires_grad_()
    w1 = (torch.randn(256, 256, 1, 1, device="cuda") * 256 ** -0.5).requires_grad_()
    gsc, g1 = _x(4, 512, 8, 8, 32), _x(4, 256, 16, 16, 33)
    before = len(hg._DEFER["pending_f32"])
    with hg.deferred_weight_grads():
        sc, y1, _ = proj_pair(x, wsc, 2, w1)
        (sc.float() * gsc.float()).sum().add((y1.float() * g1.float()).sum()).backward()
        assert len(hg._DEFER["pending_f32"]) - before == 2  # the shortcut's and conv1's
    assert hg.flush_weight_grads() >= 2
    xr = x.detach().float().requires_grad_()
    ar, br = wsc.detach().clone().requires_grad_(), w1.detach().clone().requires_grad_()
    scr = F.conv2d(xr, ar.to(torch.bfloat16).float(), stride=2)
    y1r = F.conv2d(xr, br.to(torch.bfloat16).float())
    (scr * gsc.float()).sum().add((y1r * g1.float()).sum()).backward()
    torch.testing.assert_close(sc.float(), scr, rtol=3e-2, atol=3e-2)
    for got, want in ((wsc.grad, ar.grad), (w1.grad, br.grad), (x.grad.float(), xr.grad)):
        torch.testing.assert_close(got, want, rtol=3e-2, atol=3e-2 * want.abs().max().item())
