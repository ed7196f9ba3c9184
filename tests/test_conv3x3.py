"""3x3 convolutions as implicit GEMMs on the pipelined MFMA kernel (mifx.ops.conv3x3, csrc/gemm8.hip CV 1 / CV 2):
forward (+ BatchNorm statistics), input gradient (stride 1 on the same kernel, stride 2 on the phase-split kernel),
weight gradient (deferred grouped TN with the per-tap pixel gather, and the library fallback), and the BatchNorm
coupling -- all against plain PyTorch fp32 references."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _x(n, c, h, w, seed, scale=1.0, shift=0.0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    t = (torch.randn(n, c, h, w, device="cuda", generator=g) * scale + shift).to(torch.bfloat16)
    return t.contiguous(memory_format=torch.channels_last)


def _w(cout, cin, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    w = torch.randn(cout, cin, 3, 3, device="cuda", generator=g) * (9 * cin) ** -0.5
    return w.contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("n,cin,hw,cout,stride", [(4, 128, 16, 128, 1), (4, 128, 16, 256, 1), (2, 256, 16, 128, 1),
                                                   (4, 128, 32, 128, 2), (2, 256, 16, 256, 2), (8, 512, 4, 512, 1),
                                                   (4, 256, 16, 256, 1), (8, 512, 8, 512, 2)])
def test_conv3x3_forward_stats_backward(n, cin, hw, cout, stride):
    from mifx.ops import gemm as hg
    from mifx.ops.conv3x3 import conv3x3, eligible

    x = _x(n, cin, hw, hw, 1).requires_grad_()
    w = _w(cout, cin, 2).requires_grad_()
    assert eligible(x, w, stride, 1)
    y, part = conv3x3(x, w, stride, stats=True)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == torch.bfloat16
    ref = F.conv2d(x.float(), w.to(torch.bfloat16).float(), stride=stride, padding=1)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs()
    assert (err <= 2 ** -7 * ref.abs() + 2e-2).all(), err.max().item()
    # per-tile statistics of the stored output
    M = y.shape[0] * y.shape[2] * y.shape[3]
    T = part.shape[1]
    yf = y.float().permute(0, 2, 3, 1).reshape(M, cout).double()
    tm, tm2 = part[0].double(), part[1].double()
    mean = tm.mean(0)
    var = (tm2.sum(0) + (M // T) * ((tm - mean) ** 2).sum(0)) / M
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(var, yf.var(0, unbiased=False), rtol=1e-4, atol=1e-5)
    # backward (library weight gradient: not deferring)
    gy = _x(*y.shape, 3)
    y.backward(gy)
    xr, wr = x.detach().float().requires_grad_(), w.detach().clone().requires_grad_()
    F.conv2d(xr, wr.to(torch.bfloat16).float(), stride=stride, padding=1).backward(gy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, rtol=2e-2, atol=2e-2 * xr.grad.abs().max().item())
    torch.testing.assert_close(w.grad, wr.grad, rtol=2e-2, atol=2e-2 * wr.grad.abs().max().item())
    # deferred weight gradient: the grouped TN launch gathering x per output pixel and tap (overwrite, then
    # accumulate into an existing gradient)
    deferred = cin % 256 == 0 and cout % 256 == 0  # (128-wide weight gradients stay on the library)
    for acc in (False, True):
        w2 = w.detach().clone().requires_grad_()
        if acc:
            w2.grad = torch.ones_like(w2)
        y2, _ = conv3x3(x.detach(), w2, stride)
        with hg.deferred_weight_grads():
            y2.backward(gy)
        assert hg.flush_weight_grads() == (1 if deferred else 0)
        assert w2.grad.is_contiguous(memory_format=torch.channels_last)
        torch.testing.assert_close(w2.grad, wr.grad + (1 if acc else 0), rtol=2e-2,
                                   atol=2e-2 * wr.grad.abs().max().item())


def test_conv3x3_bn_coupled_backward():
    """BatchNorm + ReLU -> 3x3 conv with bn_input=True: the BatchNorm takes its backward sums from the dX epilogue;
    gradients equal the uncoupled path's and fp32's."""
    from mifx.ops.bn_relu import BatchNormReLU2d
    from mifx.ops.conv3x3 import conv3x3

    torch.manual_seed(1)
    x0 = _x(4, 128, 16, 16, 11, 1.5, 0.3)
    w = _w(256, 128, 12)
    gy = _x(4, 256, 16, 16, 13)
    bn_ref = BatchNormReLU2d(128).cuda()
    with torch.no_grad():
        bn_ref.weight.uniform_(0.5, 1.5)
        bn_ref.bias.uniform_(-0.2, 0.2)
    grads = []
    for couple in (False, True):
        bn = copy.deepcopy(bn_ref)
        x = x0.detach().clone().requires_grad_()
        wc = w.detach().clone().requires_grad_()
        y, _ = conv3x3(bn(x), wc, 1, bn_input=couple)
        (y.float() * gy.float()).sum().backward()
        grads.append((x.grad.float(), bn.weight.grad, bn.bias.grad, wc.grad))
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2 * b.abs().max().item())
    xr = x0.detach().float().requires_grad_()
    wr = bn_ref.weight.detach().clone().requires_grad_()
    br = bn_ref.bias.detach().clone().requires_grad_()
    pre = F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5))
    (F.conv2d(pre, w.to(torch.bfloat16).float(), padding=1) * gy.float()).sum().backward()
    for a, b in zip(grads[1][:3], (xr.grad, wr.grad, br.grad)):
        torch.testing.assert_close(a, b, rtol=5e-2, atol=5e-2 * b.abs().max().item())


def test_weight_prep_images_exact():
    """One launch writes every registered weight's bf16 images: 1x1 [Cout, C] and its transpose, 3x3 [Cout, 9 C]
    (channels_last storage) and the flipped transpose [C, 9 Cout] -- bit-equal to the per-weight torch casts; a weight
    changed after the refresh has no image (stale version)."""
    from mifx.ops import weight_prep as wp

    ws = [torch.randn(256, 128, 1, 1, device="cuda"), torch.randn(128, 512, 1, 1, device="cuda"),
          torch.randn(256, 128, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last),
          torch.randn(128, 256, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)]
    prep = wp.WeightPrep(ws)
    prep.refresh()
    for w in ws:
        fwd, bwd = wp.images(w)
        cout, c = w.shape[:2]
        wb = w.to(torch.bfloat16)
        if w.shape[2] == 1:
            assert torch.equal(fwd, wb.view(cout, c))
            assert torch.equal(bwd, wb.view(cout, c).t().contiguous())
        else:
            assert torch.equal(fwd, wb.permute(0, 2, 3, 1).reshape(cout, 9 * c))
            want = wb.permute(0, 2, 3, 1).flip(1, 2).permute(3, 1, 2, 0).reshape(c, 9 * cout)
            assert torch.equal(bwd, want)
    ws[0].add_(1.0)
    assert wp.images(ws[0]) is None and wp.images(ws[1]) is not None
    prep.close()
    assert wp.images(ws[1]) is None
