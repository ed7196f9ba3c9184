"""Grouped NHWC implicit-GEMM convolution (csrc/gconv.hip) vs an fp32 PyTorch reference."""
import pytest
import torch
import torch.nn.functional as F

from mifx.ops import gconv


def test_eligibility_rules():
    x = torch.empty(2, 3 * 64, 8, 8)
    assert not gconv.eligible(x, torch.empty(3 * 128, 64, 5, 5), 3, 2)  # CPU tensor
    w = torch.empty(3 * 128, 32, 5, 5)
    assert not gconv.eligible(torch.empty(2, 96, 8, 8), w, 3, 2)


def test_cpu_falls_back_to_f_conv2d():
    torch.manual_seed(0)
    x, w, b = torch.randn(2, 6, 7, 7), torch.randn(8, 3, 3, 3), torch.randn(8)
    torch.testing.assert_close(gconv.conv2d(x, w, b, padding=1, groups=2), F.conv2d(x, w, b, padding=1, groups=2))


@pytest.mark.gpu
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("N,H,G,C,K,R,pad", [(4, 14, 3, 64, 128, 5, 2), (3, 7, 2, 64, 64, 3, 1),
                                             (2, 9, 1, 64, 64, 3, 0), (5, 6, 4, 128, 64, 5, 2),
                                             (3, 7, 2, 32, 128, 3, 1), (2, 5, 1, 128, 256, 3, 0),
                                             (6, 8, 5, 32, 64, 1, 0),
                                             # enough (tap, k, group) tiles for the HIP weight-gradient kernel
                                             (2, 6, 32, 64, 128, 5, 2), (2, 5, 96, 32, 128, 3, 1),
                                             # 32-channel output tiles (PATE inference_deeper's 96-channel layers)
                                             (3, 8, 4, 96, 96, 3, 1), (2, 7, 3, 96, 192, 3, 1),
                                             # HIP weight gradient over a tap-straddling (tap, c) column space
                                             (2, 5, 48, 96, 96, 3, 1), (2, 4, 24, 192, 192, 3, 1)])
def test_gconv_fwd_bwd_match_fp32_reference(N, H, G, C, K, R, pad, relu):
    _check_against_reference(N, H, G, C, K, R, pad, relu, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,G,C,K,R,pad", [(2, 9, 3, 96, 96, 3, 0), (2, 15, 24, 192, 192, 3, 0),
                                             (3, 8, 2, 64, 128, 3, 1)])
def test_gconv_stride2_matches_fp32_reference(N, H, G, C, K, R, pad):
    """Strided forward, phase-split input gradient and weight gradient, all on the HIP kernels -- PATE
    inference_deeper's stride-2 layers."""
    _check_against_reference(N, H, G, C, K, R, pad, False, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,G,C,K,R,pad,stride", [(2, 9, 3, 96, 96, 3, 0, 2), (2, 10, 2, 64, 32, 3, 1, 2),
                                                    (3, 11, 1, 128, 64, 5, 2, 2), (2, 13, 4, 32, 96, 3, 1, 3),
                                                    (2, 7, 2, 32, 32, 1, 0, 2), (1, 16, 250, 96, 96, 3, 0, 2)])
def test_gconv_strided_input_gradient_kernel(N, H, G, C, K, R, pad, stride):
    """The phase-split input gradient (csrc/gconv.hip gconv_dgrad_s) alone against the fp32 reference: odd and
    even sizes (phases with fewer rows), strides 2 and 3, 1x1 taps (phases without taps: zero rows), 250 groups."""
    torch.manual_seed(1)
    dev = "cuda"
    W = H + 1
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - R) // stride + 1
    w = (0.05 * torch.randn(G * K, C, R, R, device=dev)).to(torch.bfloat16)
    dy = torch.randn(N, G * K, Ho, Wo, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_input((N, G * C, H, W), w.float(), dy.float(), stride=stride, padding=pad, groups=G)
    got = gconv.dgrad_strided(dy, w, N, H, W, G, C, K, R, R, pad, stride)
    assert got.is_contiguous(memory_format=torch.channels_last)
    sc = ref.abs().max()
    torch.testing.assert_close(got.float() / sc, ref / sc, rtol=0, atol=1e-2)


def _check_against_reference(N, H, G, C, K, R, pad, relu, stride):
    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(N, G * C, H, H + 1, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (0.05 * torch.randn(G * K, C, R, R, device=dev)).to(torch.bfloat16).float()
    b = torch.randn(G * K, device=dev)
    xr, wr, br = x.float().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    ref = F.conv2d(xr, wr, br, padding=pad, groups=G, stride=stride)
    if relu:
        ref = F.relu(ref)
    xk, wk, bk = x.clone().requires_grad_(), w.clone().requires_grad_(), b.clone().requires_grad_()
    assert gconv.eligible(xk, wk, G, pad, stride)
    out = gconv.conv2d(xk, wk, bk, padding=pad, groups=G, relu=relu, stride=stride)
    assert out.dtype == torch.bfloat16 and out.is_contiguous(memory_format=torch.channels_last)
    s = ref.abs().max()
    torch.testing.assert_close(out.float() / s, ref / s, rtol=0, atol=1e-2)
    dy = torch.randn_like(ref).to(torch.bfloat16)
    ref.backward(dy.float())
    out.backward(dy)
    for got, want in ((xk.grad, xr.grad), (wk.grad, wr.grad), (bk.grad, br.grad)):
        sc = want.abs().max()
        torch.testing.assert_close(got.float() / sc, want / sc, rtol=0, atol=1.5e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,C,K,R,pad,stride", [(8, 14, 64, 64, 3, 1, 1), (4, 15, 128, 128, 3, 1, 2),
                                                  (8, 7, 256, 64, 1, 0, 1), (4, 14, 64, 256, 1, 0, 2)])
def test_single_group_pixel_split_weight_gradient(N, H, C, K, R, pad, stride):
    """G = 1 (ResNet-50's convs): few (tap, k) tiles, so the weight gradient splits the output pixels and sums the
    partials deterministically; vs the fp32 reference, and bit-identical across two runs."""
    torch.manual_seed(2)
    dev = "cuda"
    x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    Ho = (H + 2 * pad - R) // stride + 1
    dy = torch.randn(N, K, Ho, Ho, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    if R == 1:  # the 1x1 path (batched GEMM) is separate; call the kernel directly
        got = gconv.wgrad(x, dy, N, H, H, 1, C, K, R, R, pad, stride)
    else:
        got = gconv.wgrad(x, dy, N, H, H, 1, C, K, R, R, pad, stride)
    ref = torch.nn.grad.conv2d_weight(x.float(), (K, C, R, R), dy.float(), stride=stride, padding=pad)
    sc = ref.abs().max()
    torch.testing.assert_close(got / sc, ref / sc, rtol=0, atol=2e-3)
    assert torch.equal(got, gconv.wgrad(x, dy, N, H, H, 1, C, K, R, R, pad, stride))


@pytest.mark.gpu
def test_resnet_block_on_hip_convs_matches_miopen(monkeypatch):
    """A ResNet-50 v2 bottleneck (1x1 / 3x3 stride 2 / 1x1 + projection shortcut) with HipConv2d vs nn.Conv2d:
    same outputs and parameter gradients to bf16 tolerance."""
    import importlib

    import mifx.models.resnet as R

    torch.manual_seed(3)
    x = torch.randn(8, 256, 28, 28, device="cuda").contiguous(memory_format=torch.channels_last)
    outs = []
    for hip in (False, True):
        monkeypatch.setattr(R, "USE_HIP_CONV", hip)
        torch.manual_seed(4)
        blk = R.PreActBottleneck(256, 128, 2).cuda().to(memory_format=torch.channels_last)
        assert isinstance(blk.conv2, R.HipConv2d) == hip
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y, sc = blk(x)
            loss = (y.float() * sc.float()).mean()
        loss.backward()
        outs.append((y.float(), {n: p.grad.float() for n, p in blk.named_parameters()}))
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=3e-2, atol=3e-2)
    for n, g in outs[0][1].items():
        s = g.abs().max()
        torch.testing.assert_close(outs[1][1][n] / s, g / s, rtol=0, atol=3e-2, msg=n)
    _ = importlib


@pytest.mark.gpu
@pytest.mark.parametrize("C,K,H,R,stride,pad", [(512, 512, 7, 3, 1, 1), (1024, 2048, 14, 1, 2, 0),
                                                (256, 1024, 14, 1, 1, 0), (64, 64, 56, 3, 1, 1)])
def test_split_reduction_forward_batch1(C, K, H, R, stride, pad):
    """Batch-1 ResNet-50 shapes whose pixel x channel tiles cannot fill the chip: the forward splits its reduction
    over workgroups (fp32 partials added in order by gconv_splitk_finish, + bias, ReLU); against the fp32 reference,
    and deterministic run to run."""
    torch.manual_seed(7)
    x = torch.randn(1, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(K, C, R, R, device="cuda") / (C * R * R) ** 0.5).to(torch.bfloat16)
    b = torch.randn(K, device="cuda")
    ks = int(gconv._fns()["ksplit"](1, H, H, 1, C, K, R, R, pad, stride))
    if H <= 14:
        assert ks > 1
    wf = w.view(1, K, C, R, R).permute(0, 1, 3, 4, 2).contiguous()
    y = gconv._launch(x, wf, b, 1, H, H, 1, C, K, R, R, pad, True, stride)
    y2 = gconv._launch(x, wf, b, 1, H, H, 1, C, K, R, R, pad, True, stride)
    assert torch.equal(y, y2)
    ref = torch.relu(F.conv2d(x.float(), w.float(), b, stride=stride, padding=pad))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2 * float(ref.abs().max()))
