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


def _pipe():
    spec = importlib.util.spec_from_file_location("rp", os.path.join(ROOT, "examples/image/resnet_pipeline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _run_trainer(tmp_path, name, num_gpus, batch, accum, steps=3, checkpoint_every=0, device="cpu"):
    from safetensors.torch import load_file

    from mifx.orchestration import LocalDagRunner

    p = _pipe().create_pipeline(str(tmp_path / name), 48, 40, 32, 5, steps, batch, num_gpus, checkpoint_every, accum,
                                name=name)
    res = LocalDagRunner(device=device).run(p)
    assert res.succeeded
    out = res.components["ImageTrainer"].outputs["output"][0]
    md = os.path.join(out.uri, "serving_model_dir")
    ck = sorted(f for f in os.listdir(md) if f.startswith("ckpt-"))
    assert ck == [f"ckpt-{steps}.safetensors"]
    return out, load_file(os.path.join(md, ck[0]))


def test_image_trainer_dp_two_ranks_equal_one_process_accumulating(tmp_path):
    """ImageTrainer(custom_config num_gpus=2): the component launches two gloo ranks itself; each trains its half
    of every global sample with its own BatchNorm statistics and the gradients are averaged (bucket views). One
    process accumulating the same two micro-batches per step computes the same update."""
    o1, one = _run_trainer(tmp_path, "acc", 1, 4, 2)
    o2, dp = _run_trainer(tmp_path, "dp", 2, 4, 1)
    assert o2.custom_properties["num_replicas"] == 2 and o1.custom_properties["num_replicas"] == 1
    ws = [k for k in one if k.startswith("model.") and "running" not in k and "num_batches" not in k]
    assert len(ws) > 100
    for k in ws:
        np.testing.assert_allclose(dp[k].numpy(), one[k].numpy(), rtol=2e-4, atol=2e-6, err_msg=k)


def test_image_trainer_resume_equals_uninterrupted(tmp_path):
    """Checkpoint every 2 steps; a trainer restarted from the step-2 checkpoint ends with the weights, momentum
    buffers and BatchNorm statistics of an uninterrupted 4-step run."""
    from safetensors.torch import load_file

    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    imgs, labels = synthetic_imagenet(40, 40, 5, seed=3)

    def make():
        return ResNetTrainer(4, "cpu", imgs, labels, num_classes=5, warmup_steps=2, crop=32)

    a = make()
    for _ in range(4):
        a.step()
    b = make()
    for _ in range(2):
        b.step()
    path = b.save_checkpoint(str(tmp_path / "ck"))
    c = make()
    c.restore(path)
    assert c.step_idx == 2
    for _ in range(2):
        c.step()
    sa, sc = a.state_dict(), c.state_dict()
    assert set(sa) == set(sc) and any(k.startswith("opt.momentum") for k in sa)
    for k in sa:
        torch.testing.assert_close(sc[k], sa[k], rtol=0, atol=0, msg=k)
    assert load_file(path)["step"].item() == 2


@pytest.mark.gpu
def test_image_trainer_dp_shared_gpu_rehearsal(tmp_path, monkeypatch):
    """The DP component flow on one GPU: 2 ranks share cuda:0 over gloo (functional only), bf16 MIOpen path."""
    monkeypatch.setenv("MIFX_SHARED_GPU", "1")
    monkeypatch.setenv("MIFX_DIST_BACKEND", "gloo")
    out, ck = _run_trainer(tmp_path, "dpgpu", 2, 8, 1, steps=2, device="cuda")
    assert out.custom_properties["num_replicas"] == 2
    assert np.isfinite(out.custom_properties["final_loss"])
