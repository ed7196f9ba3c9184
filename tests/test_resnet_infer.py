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
