"""Fused BatchNorm+ReLU (csrc/bn_relu.hip) vs the PyTorch fp32 reference."""
import pytest
import torch
import torch.nn.functional as F

import mifx.ops.bn_relu as bnr
from mifx.ops.bn_relu import BatchNormReLU2d, bn_relu


def test_cpu_reference_path_matches_batchnorm_relu():
    torch.manual_seed(0)
    m = BatchNormReLU2d(16)
    ref = torch.nn.BatchNorm2d(16)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(4, 16, 5, 5)
    torch.testing.assert_close(m(x), F.relu(ref(x)))
    torch.testing.assert_close(m.running_var, ref.running_var)
    m.eval(), ref.eval()
    torch.testing.assert_close(m(x), F.relu(ref(x)))


def test_deferred_batch_counts_one_tensor(tmp_path):
    """defer_batch_counts: every BatchNormReLU2d's num_batches_tracked becomes an element of one tensor, forwards stop
    advancing it, one add_(1) advances all; state_dict round trip and a safetensors save of cloned entries work."""
    from safetensors.torch import load_file, save_file

    torch.manual_seed(0)
    m = torch.nn.Sequential(BatchNormReLU2d(8), torch.nn.Conv2d(8, 8, 1), BatchNormReLU2d(8))
    m(torch.randn(2, 8, 3, 3))  # one counted forward before deferring
    flat = bnr.defer_batch_counts(m)
    assert flat is not None and flat.tolist() == [1, 1]
    m(torch.randn(2, 8, 3, 3))
    assert flat.tolist() == [1, 1]  # forwards no longer count
    flat.add_(1)
    assert [int(b.num_batches_tracked) for b in (m[0], m[2])] == [2, 2]
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    save_file(sd, str(tmp_path / "m.safetensors"))
    m[0].num_batches_tracked.fill_(7)  # in place: still a view of the shared tensor
    assert flat.tolist() == [7, 2]
    m.load_state_dict(load_file(str(tmp_path / "m.safetensors")))
    assert flat.tolist() == [2, 2]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 3e-2)])
@pytest.mark.parametrize("shape", [(4, 64, 14, 14), (8, 256, 7, 7), (2, 2048, 3, 3), (3, 24, 5, 7)])
def test_fused_bn_relu_matches_fp32_reference(dtype, tol, shape):
    torch.manual_seed(0)
    N, C, H, W = shape
    x = (torch.randn(shape, device="cuda") * 2 + 0.5).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_()
    b = (torch.randn(C, device="cuda") * 0.2).requires_grad_()
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    xg = x.detach().requires_grad_()
    y = bn_relu(xg, w, b, rm, rv, True, 0.1, 1e-5)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == dtype
    x32 = x.detach().float().requires_grad_()
    w2, b2 = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    rm2, rv2 = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    ref = F.relu(F.batch_norm(x32, rm2, rv2, w2, b2, True, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), ref, rtol=tol, atol=tol)
    torch.testing.assert_close(rm, rm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rv, rv2, rtol=1e-4, atol=1e-5)
    g = torch.randn_like(ref)
    y.backward(g.to(dtype).contiguous(memory_format=torch.channels_last))
    ref.backward(g)
    torch.testing.assert_close(xg.grad.float(), x32.grad, rtol=tol * 3, atol=tol * 3)
    m = N * H * W
    torch.testing.assert_close(w.grad, w2.grad, rtol=tol * 3, atol=tol * 3 * m ** 0.5)
    torch.testing.assert_close(b.grad, b2.grad, rtol=tol * 3, atol=tol * 3 * m ** 0.5)
    # eval path (running statistics)
    ye = bn_relu(x, w.detach(), b.detach(), rm, rv, False, 0.1, 1e-5)
    re = F.relu(F.batch_norm(x.float(), rm, rv, w.detach(), b.detach(), False, 0.1, 1e-5))
    torch.testing.assert_close(ye.float(), re, rtol=tol, atol=tol)


@pytest.mark.gpu
def test_fused_bn_relu_is_deterministic():
    torch.manual_seed(1)
    x = torch.randn(16, 128, 28, 28, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.ones(128, device="cuda", requires_grad=True)
    b = torch.zeros(128, device="cuda", requires_grad=True)
    outs = []
    for _ in range(2):
        xg = x.detach().requires_grad_()
        y = bn_relu(xg, w, b, None, None, True)
        y.sum().backward()
        outs.append((y.detach().clone(), xg.grad.clone(), w.grad.clone()))
        w.grad = None
        b.grad = None
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


def test_cpu_add_bn_relu_reference():
    from mifx.ops.bn_relu import add_bn_relu

    a, b = torch.randn(2, 8, 3, 3), torch.randn(2, 8, 3, 3)
    w, bias = torch.ones(8), torch.zeros(8)
    y, s = add_bn_relu(a, b, w, bias, None, None, True)
    torch.testing.assert_close(s, a + b)
    torch.testing.assert_close(y, F.relu(F.batch_norm(a + b, None, None, w, bias, True)))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 3e-2)])
def test_fused_add_bn_relu_matches_reference(dtype, tol):
    from mifx.ops.bn_relu import add_bn_relu

    torch.manual_seed(0)
    shape = (4, 256, 14, 14)
    C = shape[1]
    mk = lambda: torch.randn(shape, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)  # noqa
    a, b = mk().requires_grad_(), mk().requires_grad_()
    w = (torch.rand(C, device="cuda") + 0.5).requires_grad_()
    bias = (torch.randn(C, device="cuda") * 0.2).requires_grad_()
    y, s = add_bn_relu(a, b, w, bias, None, None, True)
    a32, b32 = a.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    w2, bias2 = w.detach().clone().requires_grad_(), bias.detach().clone().requires_grad_()
    s_ref = (a32 + b32).to(dtype).float()  # the fused kernel normalises the stored (rounded) sum
    s_ref = a32 + b32 + (s_ref - (a32 + b32)).detach()
    y_ref = F.relu(F.batch_norm(s_ref, None, None, w2, bias2, True, 0.1, 1e-5))
    torch.testing.assert_close(s.float(), s_ref, rtol=tol, atol=tol)
    torch.testing.assert_close(y.float(), y_ref, rtol=tol, atol=tol)
    gy, gs = torch.randn_like(y_ref), torch.randn_like(y_ref)
    torch.autograd.backward([y, s], [gy.to(dtype).contiguous(memory_format=torch.channels_last),
                                     gs.to(dtype).contiguous(memory_format=torch.channels_last)])
    torch.autograd.backward([y_ref, s_ref], [gy, gs])
    torch.testing.assert_close(a.grad.float(), a32.grad, rtol=tol * 3, atol=tol * 3)
    torch.testing.assert_close(b.grad.float(), b32.grad, rtol=tol * 3, atol=tol * 3)
    m = shape[0] * shape[2] * shape[3]
    torch.testing.assert_close(w.grad, w2.grad, rtol=tol * 3, atol=tol * 3 * m ** 0.5)


@pytest.mark.gpu
def test_resnet_fused_blocks_match_fp64_reference():
    """Pre-activation ResNet (every bottleneck kind: conv shortcut, stride 2, fused residual add) with
    the fused BN kernels in fp32 vs the same weights in fp64 on the PyTorch path, per-parameter relative
    Frobenius error of every gradient.

    The tight check is against the same network with PyTorch BN + ReLU on the same NHWC convolutions
    (run first, so both use the same MIOpen solvers); fp64 is a loose sanity bound, because MIOpen's
    solver choice for a first-seen fp32 NHWC problem can be a reduced-precision one (measured 3e-3 on
    the stem's weight gradient when the fused model ran first).
    Conditioning notes (one-off fp64 gradient and model-divergence probes on MI355X, round 2):
    (1) the full 16-block net at 64x64 / batch 4 has train-mode BN over as few as 16 samples per
    channel and its gradients are noise-dominated even for the fp32 PyTorch path (1-3 % vs fp64), so a
    one-block-per-stage net is used; (2) MIOpen's reduced-precision (xf32) convolution solvers are
    selected while `allow_tf32` is on (~3e-3 gradient error on both the PyTorch and the fused path), so
    the check runs with it off. Measured: fused 3.6e-6 vs PyTorch fp32 3.3e-6 global rel. error."""
    import copy

    from mifx.models.resnet import ResNetV2

    saved = torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32
    torch.backends.cudnn.allow_tf32 = torch.backends.cuda.matmul.allow_tf32 = False
    try:
        torch.manual_seed(0)
        m = ResNetV2((1, 1, 1, 1), 10).cuda()
        x = torch.rand(8, 3, 64, 64, device="cuda")
        xl = x.contiguous(memory_format=torch.channels_last)
        gout = torch.randn(8, 10, device="cuda")
        m64 = copy.deepcopy(m).double()
        out64 = m64(x.double())
        out64.backward(gout.double())
        # same NHWC convolutions (same MIOpen solvers, chosen on this first run), PyTorch BN + ReLU
        mr = copy.deepcopy(m).to(memory_format=torch.channels_last)
        real_ok = bnr.native_ok
        bnr.native_ok = lambda t: False
        try:
            out_r = mr(xl)
            out_r.backward(gout)
        finally:
            bnr.native_ok = real_ok
        mf = copy.deepcopy(m).to(memory_format=torch.channels_last)
        out = mf(xl)  # fused native path (fp32)
        out.backward(gout)
    finally:
        torch.backends.cudnn.allow_tf32, torch.backends.cuda.matmul.allow_tf32 = saved
    torch.testing.assert_close(out.double(), out64, rtol=1e-4, atol=1e-4)
    g64, gr = dict(m64.named_parameters()), dict(mr.named_parameters())

    def rel(a, b):
        return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()

    rows = [(n, rel(p.grad, gr[n].grad), rel(p.grad, g64[n].grad), rel(gr[n].grad, g64[n].grad))
            for n, p in mf.named_parameters()]
    table = "\n".join(f"  {n}: fused~torch {a:.2e}  fused~fp64 {b:.2e}  torch~fp64 {c:.2e}" for n, a, b, c in rows)
    # Tight check where the gradient reaches the parameter through our kernels only (post-BN, fc and the
    # last block's BN+ReLU layers, whose incoming gradients come from the fused BN / fc path): fused vs
    # the PyTorch-BN fp32 path. Upstream of a MIOpen backward-data convolution the two fp32 runs feed the
    # convolution gradients in different layouts, and on some machines MIOpen then picks a solver with
    # ~3e-3 relative error for the fused run only (measured: every parameter upstream of blocks.2.conv2's
    # dgrad at 2-5e-3 vs fp64 while the PyTorch run is at 3e-6, identically with two BN kernel versions);
    # there only the loose fp64 bound applies. The BN kernels themselves are checked tightly above.
    tight = ("post_bn.", "fc.", "blocks.3.bn2.", "blocks.3.bn1.")
    for n, a, b, c in rows:
        if n.startswith(tight):
            assert a < 1e-4, f"{n}: fused vs PyTorch-BN relative gradient error {a:.2e}\n{table}"
        assert b < 1e-2, f"{n}: fused vs fp64 relative gradient error {b:.2e}\n{table}"


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (2, 16, 8, 6), (3, 16, 9, 7), (2, 8, 1, 1)])
def test_maxpool3s2_matches_pytorch(shape):
    """HIP 3x3/s2/p1 NHWC max-pool (1-byte argmax, gather backward) vs F.max_pool2d: identical forward, and
    the backward equal to PyTorch's (ties are avoided by distinct values so both pick the same position)."""
    from mifx.ops.pool import max_pool3s2, native_ok

    torch.manual_seed(0)
    N, C, H, W = shape
    vals = torch.randperm(N * C * H * W, device="cuda").float() / (N * C * H * W)  # distinct, bf16-exact steps
    x = (vals.view(N, C, H, W) * 256).round().bfloat16().contiguous(memory_format=torch.channels_last)
    x = x + torch.randn_like(x.float()).mul(1e-3).bfloat16()  # break most bf16 ties
    assert native_ok(x)
    xa = x.detach().requires_grad_()
    xb = x.detach().float().requires_grad_()
    ya = max_pool3s2(xa)
    yb = torch.nn.functional.max_pool2d(xb, 3, 2, 1)
    assert ya.shape == yb.shape and ya.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(ya.float(), yb, rtol=0, atol=0)
    g = torch.randn_like(yb).bfloat16().float()
    ya.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    yb.backward(g)
    # the kernel rounds each input gradient (a sum of <= 4 window gradients) to bf16 once: compare against the
    # fp32 reference rounded the same way. Positions that are an exact bf16 tie may route to a different tap
    # than PyTorch's, so require exact equality almost everywhere rather than everywhere.
    ref = xb.grad.bfloat16().float()
    same = xa.grad.float() == ref
    assert same.float().mean() > 0.999, f"{(~same).sum().item()} of {same.numel()} input gradients differ"


@pytest.mark.gpu
def test_fused_bn_large_mean_variance_vs_fp64():
    """Channels whose mean dwarfs their std (mean 100, std 1, e.g. residual sums): the shifted-sum statistics
    must match an fp64 reference (E[x^2]-E[x]^2 from fp32 partials loses ~all digits of the variance here)."""
    torch.manual_seed(5)
    C = 64
    x = (torch.randn(8, C, 16, 16, device="cuda") + 100.0 + torch.arange(C, device="cuda").view(1, C, 1, 1))
    x = x.contiguous(memory_format=torch.channels_last)
    w, b = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y = bn_relu(x, w, b, rm, rv, True, 1.0, 1e-5, relu=False)  # momentum 1: running stats = batch stats
    x64 = x.double()
    var64 = x64.var(dim=(0, 2, 3), unbiased=False)
    ref = (x64 - x64.mean(dim=(0, 2, 3), keepdim=True)) / (var64.view(1, C, 1, 1) + 1e-5).sqrt()
    torch.testing.assert_close(y.double(), ref, rtol=0, atol=2e-3)
    torch.testing.assert_close(rv.double(), x64.var(dim=(0, 2, 3), unbiased=True), rtol=2e-3, atol=0)
    torch.testing.assert_close(rm.double(), x64.mean(dim=(0, 2, 3)), rtol=1e-6, atol=0)


@pytest.mark.gpu
def test_maxpool3s2_nan_routing_matches_pytorch():
    """Several NaNs in one window: forward NaN and the gradient routed to the LAST NaN (PyTorch's rule)."""
    from mifx.ops.pool import max_pool3s2

    x = torch.randn(1, 8, 6, 6, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    x[0, :, 1, 1] = float("nan")
    x[0, :, 1, 2] = float("nan")
    x[0, :, 4, 3] = float("nan")
    xa = x.detach().requires_grad_()
    xb = x.detach().float().requires_grad_()
    ya = max_pool3s2(xa)
    yb = torch.nn.functional.max_pool2d(xb, 3, 2, 1)
    assert torch.equal(torch.isnan(ya.float()), torch.isnan(yb))
    g = torch.ones_like(yb)
    ya.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    yb.backward(g)
    torch.testing.assert_close(xa.grad.float(), xb.grad, rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(2, 64, 28, 28), (3, 16, 14, 14), (2, 8, 7, 9)])
def test_maxpool3s2_tf_same_matches_padded_pytorch(shape):
    """TF-SAME 3x3/2 pooling of the PATE CNN (asymmetric padding) on the HIP kernels == F.max_pool2d over the
    -inf-padded input, forward and backward."""
    import math

    from mifx.models.cnn import _same_pad
    from mifx.ops.pool import max_pool3s2_same

    torch.manual_seed(1)
    N, C, H, W = shape
    vals = torch.randperm(N * C * H * W, device="cuda").float() / (N * C * H * W)
    x = (vals.view(N, C, H, W) * 256).round().bfloat16().contiguous(memory_format=torch.channels_last)
    xa = x.detach().requires_grad_()
    xb = x.detach().float().requires_grad_()
    ya = max_pool3s2_same(xa)
    yb = torch.nn.functional.max_pool2d(_same_pad(xb, 3, 2, value=-math.inf), 3, 2)
    assert ya is not None and ya.shape == yb.shape
    torch.testing.assert_close(ya.float(), yb, rtol=0, atol=0)
    g = torch.randn_like(yb).bfloat16().float()
    ya.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    yb.backward(g)
    same = xa.grad.float() == xb.grad.bfloat16().float()
    assert same.float().mean() > 0.999


@pytest.mark.gpu
def test_maxpool3s2_same_fused_relu_matches_relu_then_pool():
    """relu + TF-SAME 3x3/2 pool in one kernel == F.relu then the padded F.max_pool2d, forward and backward
    (negative-only windows pass no gradient)."""
    import math

    from mifx.models.cnn import _same_pad
    from mifx.ops.pool import max_pool3s2_same

    torch.manual_seed(2)
    N, C, H, W = 2, 16, 28, 28
    vals = torch.randperm(N * C * H * W, device="cuda").float() / (N * C * H * W) - 0.7  # mostly negative
    x = (vals.view(N, C, H, W) * 256).round().bfloat16().contiguous(memory_format=torch.channels_last)
    xa = x.detach().requires_grad_()
    xb = x.detach().float().requires_grad_()
    ya = max_pool3s2_same(xa, relu=True)
    yb = torch.nn.functional.max_pool2d(_same_pad(torch.relu(xb), 3, 2, value=-math.inf), 3, 2)
    torch.testing.assert_close(ya.float(), yb, rtol=0, atol=0)
    g = torch.randn_like(yb).bfloat16().float()
    ya.backward(g.bfloat16().contiguous(memory_format=torch.channels_last))
    yb.backward(g)
    torch.testing.assert_close(xa.grad.float(), xb.grad.bfloat16().float(), rtol=0, atol=0)
