"""Direct fp32 conv kernels (csrc/conv_small.hip) against PyTorch's fp32 CPU convolution: forward, input, weight and
bias gradients for the reference's small-CNN layer shapes, plus the model classes that use them."""
import pytest
import torch
import torch.nn.functional as F

from mifx.ops import conv_small


def test_same_split_matches_tf_same():
    for h, k, s in [(28, 8, 2), (28, 3, 1), (14, 5, 1), (7, 3, 2), (28, 4, 2)]:
        ph, pw, extra = conv_small.same_split(h, h, k, s)
        total = ph * 2 + extra[3]
        out = (h + total - k) // s + 1
        assert out == -(-h // s)
        assert extra[1] == extra[3] and extra[1] in (0, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("N,C,H,K,R,stride,pad", [
    (16, 1, 28, 8, 3, 2, 0),     # Fashion-MNIST Conv8 3x3 s2
    (8, 1, 28, 32, 3, 1, 0),     # TPU CNN conv1
    (8, 32, 13, 64, 3, 1, 0),    # TPU CNN conv2
    (8, 64, 5, 64, 3, 1, 0),     # TPU CNN conv3
    (8, 1, 28, 16, 8, 2, 3),     # DP-SGD MNIST conv1 (symmetric part of SAME)
    (8, 16, 13, 32, 4, 2, 0),    # DP-SGD MNIST conv2
    (4, 3, 32, 64, 5, 1, 2),     # PATE conv1 on SVHN-shaped input
    (3, 5, 17, 7, 5, 3, 2),      # odd sizes, stride 3
])
def test_direct_conv_matches_fp32_reference(N, C, H, K, R, stride, pad):
    g = torch.Generator().manual_seed(N * 131 + K)
    x = torch.randn(N, C, H, H, generator=g)
    w = torch.randn(K, C, R, R, generator=g) * (C * R * R) ** -0.5
    b = torch.randn(K, generator=g)
    dy_shape = F.conv2d(x, w, b, stride, pad).shape
    dy = torch.randn(dy_shape, generator=g)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, stride, pad)
    yr.backward(dy)
    xg, wg, bg = (t.cuda().requires_grad_() for t in (x, w, b))
    y = conv_small.conv2d(xg, wg, bg, stride, pad)  # the kernels directly (any channel count)
    y.backward(dy.cuda())
    for got, ref in ((y, yr), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)):
        torch.testing.assert_close(got.detach().cpu(), ref.detach(), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_small_cnn_models_match_cpu(monkeypatch):
    from mifx.models.cnn import FashionCNN, MnistDPCNN, TpuMnistCNN

    monkeypatch.setenv("MIFX_SMALL_CONV", "1")
    for cls in (FashionCNN, TpuMnistCNN, MnistDPCNN):
        torch.manual_seed(0)
        m = cls().eval()
        if hasattr(m, "p"):
            m.p = 0.0
        x = torch.rand(4, 28, 28)
        ref = m(x)
        got = m.cuda()(x.cuda()).cpu()
        torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4)


def test_fashion_prefers_direct_conv_by_default(monkeypatch):
    """Per-model policy: FashionCNN's conv is on the direct kernels unless MIFX_SMALL_CONV=0; the others opt in."""
    from mifx.models.cnn import FashionCNN, MnistDPCNN
    from mifx.ops import conv_small

    monkeypatch.delenv("MIFX_SMALL_CONV", raising=False)
    assert FashionCNN().conv.prefer and not MnistDPCNN().conv1.prefer
    x = torch.zeros(2, 1, 28, 28)
    w = torch.zeros(8, 1, 3, 3)
    # (CPU tensors are never eligible; the switch logic is what is checked here)
    assert not conv_small.eligible(x, w, prefer=True)
    monkeypatch.setenv("MIFX_SMALL_CONV", "0")
    assert not conv_small.eligible(x, w, prefer=True)


@pytest.mark.gpu
def test_fashion_default_runs_direct_kernel(monkeypatch):
    from mifx.models.cnn import FashionCNN
    from mifx.ops import conv_small

    monkeypatch.delenv("MIFX_SMALL_CONV", raising=False)
    m = FashionCNN().cuda()
    x = torch.rand(4, 1, 28, 28, device="cuda")
    assert conv_small.eligible(x, m.conv.weight, prefer=m.conv.prefer)
    ref = torch.nn.functional.conv2d(x, m.conv.weight, m.conv.bias, 2)
    torch.testing.assert_close(m.conv(x), ref, rtol=1e-4, atol=1e-4)
