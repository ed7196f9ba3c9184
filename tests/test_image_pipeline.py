"""Image pipeline (ResNet-50, BASELINE config 5): crop/flip/normalize kernel semantics and the
ExampleGen -> Transform -> Trainer pipeline at toy size on CPU."""
import importlib.util
import os

import numpy as np
import pytest
import torch

from mifx.ops.image_ops import crop_flip_normalize, crop_params

ROOT = os.path.dirname(os.path.dirname(__file__))


def test_crop_params_and_reference_semantics():
    imgs = torch.randint(0, 255, (4, 40, 48, 3), dtype=torch.uint8)
    idx = torch.tensor([2, 0, 3])
    oy, ox, flip = crop_params(3, 40, 48, 32, 32, True, seed=5, step=9)
    assert ((0 <= oy) & (oy <= 8)).all() and ((0 <= ox) & (ox <= 16)).all() and set(flip) <= {0, 1}
    x = crop_flip_normalize(imgs, idx, (32, 32), True, 5, 9, mean=(0, 0, 0), std=(1, 1, 1), dtype=torch.float32)
    for b in range(3):
        ref = imgs[idx[b], oy[b]:oy[b] + 32, ox[b]:ox[b] + 32].float() / 255
        if flip[b]:
            ref = ref.flip(1)
        torch.testing.assert_close(x[b].permute(1, 2, 0), ref)
    ev = crop_flip_normalize(imgs, idx, (32, 32), False, mean=(0, 0, 0), std=(1, 1, 1), dtype=torch.float32)
    torch.testing.assert_close(ev[0].permute(1, 2, 0), imgs[2, 4:36, 8:40].float() / 255)


def test_image_pipeline_cpu(tmp_path):
    spec = importlib.util.spec_from_file_location("rp", os.path.join(ROOT, "examples/image/resnet_pipeline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    res = mod.main(["--root", str(tmp_path), "--num-images", "48", "--image-size", "40", "--crop", "32",
                    "--classes", "5", "--steps", "2", "--batch", "4", "--device", "cpu"])
    assert res.succeeded if hasattr(res, "succeeded") else True
    exports = [os.path.join(r, d) for r, ds, _ in os.walk(tmp_path) for d in ds if d == "1"]
    assert any(os.path.exists(os.path.join(e, "saved_model.json")) for e in exports)
    from mifx.serving.saved_model import load

    e = next(e for e in exports if os.path.exists(os.path.join(e, "saved_model.json")))
    out = load(e, "cpu").predict(np.random.rand(2, 3, 32, 32).astype(np.float32))["scores"]
    assert out.shape == (2, 5)


@pytest.mark.gpu
def test_crop_flip_normalize_gpu_matches_host():
    imgs = torch.randint(0, 255, (16, 64, 72, 3), dtype=torch.uint8)
    idx = torch.randint(0, 16, (9,))
    for train in (True, False):
        for dtype, tol in ((torch.float32, 1e-6), (torch.bfloat16, 1e-2)):
            h = crop_flip_normalize(imgs, idx, (56, 56), train, 3, 11, dtype=dtype)
            d = crop_flip_normalize(imgs.cuda(), idx.cuda(), (56, 56), train, 3, 11, dtype=dtype)
            assert d.is_contiguous(memory_format=torch.channels_last)
            torch.testing.assert_close(d.float().cpu(), h.float(), rtol=tol, atol=tol)


@pytest.mark.gpu
def test_resnet_trainer_gpu_steps():
    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    imgs, labels = synthetic_imagenet(128, 64, 10, device="cuda")
    tr = ResNetTrainer(32, "cuda", imgs, labels, num_classes=10, warmup_steps=1, crop=56)
    losses = [float(tr.step()) for _ in range(3)]
    assert all(np.isfinite(losses))
