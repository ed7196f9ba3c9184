"""ResNet-50 stem convolution (7x7 / 2, 3 -> 64) on csrc/stem_conv.hip vs fp32 PyTorch (forward) and the weight
gradient through the op (MIOpen), plus the CPU fallback."""
import pytest
import torch
import torch.nn.functional as F

from mifx.ops import stem


def test_stem_cpu_fallback_is_conv2d():
    x = torch.randn(2, 3, 17, 20)
    w = torch.randn(64, 3, 7, 7)
    assert not stem.eligible(x, w)
    torch.testing.assert_close(stem.stem_conv(x, w), F.conv2d(x, w, None, 2, 3))


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w_,cl", [(2, 224, 224, False), (2, 224, 224, True), (3, 65, 47, True), (1, 8, 9, False)])
def test_stem_forward_matches_fp32(n, h, w_, cl):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(n, 3, h, w_, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 3, 7, 7, device=dev, generator=g) * 0.05
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    assert stem.eligible(x, w)
    y = stem.stem_conv(x, w)
    assert y.shape == (n, 64, (h - 1) // 2 + 1, (w_ - 1) // 2 + 1) and y.is_contiguous(memory_format=torch.channels_last)
    ref = F.conv2d(x.float(), w.to(torch.bfloat16).float(), None, 2, 3)
    err = float((y.float() - ref).norm() / ref.norm())
    assert err < 5e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w_,cl", [(4, 32, 32, True), (2, 224, 224, True), (3, 45, 38, False), (300, 16, 16, True)])
def test_stem_weight_gradient(n, h, w_, cl):
    """The hand-written weight gradient (kernel-row taps, per-workgroup partials) vs fp32, both weight layouts, small
    batches split over row ranges and a batch above 256 workgroups."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, 3, h, w_, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = torch.randn(64, 3, 7, 7, device=dev, generator=g) * 0.05
    if cl:
        w = w.contiguous(memory_format=torch.channels_last)
    w.requires_grad_()
    y = stem.stem_conv(x, w)
    dy = torch.randn_like(y.float())
    y.float().backward(dy)
    wf = w.detach().to(torch.bfloat16).float().requires_grad_()
    F.conv2d(x.float(), wf, None, 2, 3).backward(dy)
    assert w.grad.dtype == torch.float32 and w.grad.shape == w.shape
    assert float((w.grad - wf.grad).norm() / wf.grad.norm()) < 1e-2
    # deterministic: the same gradient again, bit for bit
    g1 = w.grad.clone()
    w.grad = None
    stem.stem_conv(x, w).float().backward(dy)
    assert torch.equal(w.grad, g1)
