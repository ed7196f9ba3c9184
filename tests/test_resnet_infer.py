"""ResNet-50 v2 inference with the BatchNorms folded into the convolutions (mifx.models.resnet_infer):
the folding against the eval-mode network in fp32 on the CPU; the HIP path (folded conv + bias + ReLU epilogues,
residual-sum BN apply) and its captured hipGraph on the GPU."""
import copy

import pytest
import torch
import torch.nn as nn

from mifx.models.resnet import resnet50_v2
from mifx.models.resnet_infer import FoldedResNetV2


def _model(classes=10, seed=0):
    torch.manual_seed(seed)
    m = resnet50_v2(classes)
    with torch.no_grad():  # non-trivial frozen statistics, so the folding is actually exercised
        for mod in m.modules():
            if isinstance(mod, nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.5, 0.5)
                mod.running_var.uniform_(0.5, 2.0)
                mod.weight.uniform_(0.5, 1.5)
                mod.bias.uniform_(-0.2, 0.2)
    return m.eval()


def test_folded_matches_eval_model_cpu():
    m = _model()
    x = torch.rand(2, 3, 64, 64)
    with torch.no_grad():
        ref = m(x)
        got = FoldedResNetV2(m)(x)
    torch.testing.assert_close(got, ref, rtol=1e-4, atol=1e-4 * float(ref.abs().max()))


@pytest.mark.gpu
def test_folded_gpu_matches_fp32_and_graph_replays():
    m = _model(1001, seed=1)
    x = torch.rand(1, 3, 224, 224)
    with torch.no_grad():
        ref = copy.deepcopy(m).float()(x)
        mg = m.cuda().to(memory_format=torch.channels_last).eval()
        xg = x.cuda().contiguous(memory_format=torch.channels_last)
        f = FoldedResNetV2(mg)
        got = f(xg)
        rel = float((got.cpu() - ref).norm() / ref.norm())
        assert rel < 0.05, rel
        run = f.graphed(xg)
        x2 = torch.rand(1, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)
        out_g = run(x2)
        out_e = f(x2)
        torch.testing.assert_close(out_g, out_e, rtol=0, atol=1e-5 * float(out_e.abs().max()))


@pytest.mark.gpu
@pytest.mark.parametrize("N,H,C,K", [(1, 7, 512, 2048), (4, 28, 128, 512)])
def test_residual_epilogue_matches_separate_kernels(N, H, C, K):
    """csrc/gconv.hip ResEpi (conv + residual sum + the next BatchNorm + ReLU in the conv's epilogue) equals the
    separate conv, add and BN-apply kernels bit for bit -- with a split reduction (batch 1) and without."""
    from mifx.models.resnet_infer import _bn_add_relu
    from mifx.ops import gconv

    torch.manual_seed(3)
    cl = torch.channels_last
    x = torch.randn(N, C, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5).to(torch.bfloat16)
    wf = w.view(1, K, C, 1, 1).permute(0, 1, 3, 4, 2).contiguous()
    res = torch.randn(N, K, H, H, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    scale, shift = torch.rand(K, device="cuda") + 0.5, torch.randn(K, device="cuda") * 0.1
    s, y2 = gconv.launch_res(x, wf, None, N, H, H, 1, C, K, 1, 1, 0, 1, res, scale, shift)
    y = gconv._launch(x, wf, None, N, H, H, 1, C, K, 1, 1, 0, False, 1)
    y2_ref, s_ref = _bn_add_relu(y, res, scale, shift)
    assert torch.equal(s, s_ref) and torch.equal(y2, y2_ref)
