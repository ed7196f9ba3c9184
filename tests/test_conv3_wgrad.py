"""Hand-written 3x3 weight gradient (csrc/conv3_wgrad.hip) vs a PyTorch fp32 reference."""
import pytest
import torch

from mifx.ops import conv3_wgrad


def test_cpu_not_eligible():
    x = torch.randn(1, 64, 8, 8).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(1, 64, 8, 8).bfloat16().contiguous(memory_format=torch.channels_last)
    assert not conv3_wgrad.eligible(x, dy, torch.randn(64, 64, 3, 3), 1)


def _ref(x, dy, stride):
    torch.backends.cudnn.allow_tf32 = False  # a true fp32 reference
    xf = x.float().requires_grad_(False)
    w = torch.zeros(dy.shape[1], x.shape[1], 3, 3, device=x.device, requires_grad=True)
    torch.nn.functional.conv2d(xf, w, None, stride, 1).backward(dy.float())
    return w.grad


@pytest.mark.gpu
@pytest.mark.parametrize("n,c,h,w,cout,stride,cl", [
    (4, 64, 56, 56, 64, 1, True),      # ResNet-50 stage 1 (batch cut)
    (4, 128, 28, 28, 128, 1, True),    # stage 2
    (4, 128, 56, 56, 128, 2, True),    # stage 2, first block
    (2, 64, 9, 7, 128, 1, False),      # odd sizes, contiguous weight
    (3, 128, 15, 13, 64, 2, False),
    (1, 192, 5, 40, 64, 1, True),      # chunks of one row, three input slices
])
def test_conv3_wgrad_vs_fp32(n, c, h, w, cout, stride, cl):
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(11)
    oh, ow = (h - 1) // stride + 1, (w - 1) // stride + 1
    x = torch.randn(n, c, h, w, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    dy = torch.randn(n, cout, oh, ow, device=dev, generator=g).bfloat16().contiguous(
        memory_format=torch.channels_last)
    wt = torch.empty(cout, c, 3, 3, device=dev)
    if cl:
        wt = wt.contiguous(memory_format=torch.channels_last)
    assert conv3_wgrad.eligible(x, dy, wt, stride, route=False)
    dw = conv3_wgrad.wgrad(x, dy, wt, stride)
    assert dw.shape == wt.shape and dw.stride() == wt.stride() and dw.dtype == torch.float32
    ref = _ref(x, dy, stride)
    err = float((dw - ref).norm() / ref.norm())
    assert err < 1e-4, err  # fp32 accumulation of exact bf16 products: only summation order differs
    assert torch.equal(conv3_wgrad.wgrad(x, dy, wt, stride), dw)  # deterministic


@pytest.mark.gpu
def test_conv3x3_routes_weight_grad_to_kernel():
    """ResNet's 3x3 op sends a 64-channel weight gradient to the kernel (counted native) and matches fp32."""
    from mifx.ops import conv3x3, native_stats

    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(2, 64, 16, 16, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 64, 3, 3, device=dev, generator=g) * 0.05).contiguous(memory_format=torch.channels_last)
    w.requires_grad_(True)
    if not conv3x3.eligible(x, w, 1, 1):
        pytest.skip("shape not on the implicit-GEMM forward")
    native_stats.reset()
    y, _ = conv3x3.conv3x3(x, w, 1)
    dy = torch.randn(y.shape, device=dev, generator=g).bfloat16().contiguous(memory_format=torch.channels_last)
    y.backward(dy)
    ref = _ref(x, dy, 1)
    assert float((w.grad - ref).norm() / ref.norm()) < 1e-4
