"""PATE-2017 training flow: batching, whitening, EMA checkpoints, teachers -> noisy-max -> student."""
import math

import numpy as np
import pytest
import torch

from mifx.privacy.pate import deep_cnn, train_student, train_teachers


def test_batch_indices_wraps_back():
    assert deep_cnn.batch_indices(0, 10, 4) == (0, 4)
    assert deep_cnn.batch_indices(2, 10, 4) == (6, 10)  # shifted back to stay full


def test_image_whitening_matches_definition():
    rng = np.random.default_rng(0)
    x = rng.random((5, 4, 4, 3)).astype(np.float32)
    x[2] = 0.5  # constant image: std 0 -> divisor 1/sqrt(48)
    w = deep_cnn.image_whitening(x)
    for i in range(5):
        d = x[i] - x[i].mean()
        np.testing.assert_allclose(w[i], d / max(1 / math.sqrt(48), d.std()), rtol=1e-5, atol=1e-6)


def test_partition_is_disjoint_floor():
    d = np.arange(103)
    parts = [deep_cnn.partition_dataset(d, d, 10, t)[0] for t in range(10)]
    assert all(len(p) == 10 for p in parts)
    assert len(np.unique(np.concatenate(parts))) == 100


def test_checkpoint_holds_ema_shadow(tmp_path):
    x, y, _, _ = deep_cnn.load_dataset("mnist", train_size=256, test_size=16)
    cfg = deep_cnn.DeepCNNConfig(max_steps=3, batch_size=64, nb_teachers=1, ckpt_every=1000)
    deep_cnn.train(x, y, str(tmp_path / "m.ckpt"), cfg, device="cpu", log=lambda *_: None)
    ck = torch.load(str(tmp_path / "m.ckpt-2"), weights_only=True)
    # after 3 steps decay=min(.9999,(1+s)/(10+s)) is small: EMA differs from the raw weights but
    # lies between the init and the final weights for a scalar bias
    name = "out.bias"
    assert not torch.equal(ck["ema"][name], ck["state_dict"][name])
    p = deep_cnn.softmax_preds(x[:8], str(tmp_path / "m.ckpt-2"), cfg, device="cpu")
    assert p.shape == (8, 10) and np.allclose(p.sum(1), 1, atol=1e-5)


def test_teachers_student_end_to_end(tmp_path):
    common = ["--dataset", "mnist", "--train_dir", str(tmp_path), "--train_size", "900", "--test_size", "400",
              "--max_steps", "40", "--device", "cpu", "--batch_size", "64"]
    for t in range(3):
        assert train_teachers.main(common + ["--nb_teachers", "3", "--teacher_id", str(t)]) > 0.5
    acc = train_student.main(common + ["--nb_teachers", "3", "--teachers_dir", str(tmp_path), "--data_dir",
                                       str(tmp_path), "--teachers_max_steps", "40", "--stdnt_share", "200",
                                       "--lap_scale", "0", "--save_labels"])
    assert acc > 0.5
    assert (tmp_path / "mnist_3_student_clean_votes_lap_0.npy").exists()


def _states_close(pa, pb, rtol=1e-4, atol=1e-5):
    assert pa.keys() == pb.keys()
    for k in pa:
        torch.testing.assert_close(pa[k], pb[k], rtol=rtol, atol=atol, msg=k)


@pytest.mark.parametrize("deeper", [False, True])
def test_ensemble_trains_each_teacher_like_the_sequential_trainer(tmp_path, deeper):
    """ensemble.train_ensemble (all teachers as one grouped network) == deep_cnn.train per shard: same weights,
    same EMA shadow, same checkpoint files, same predictions."""
    T = 2
    x, y, xte, _ = deep_cnn.load_dataset("mnist", train_size=T * 48, test_size=16)
    # the synthetic images are clipped to [0, 1]: jitter them so no max-pool window holds exact ties (CPU max-pool
    # breaks ties differently for the ensemble's channels-last tensors than for the sequential NCHW ones); run in
    # fp64 so that the two (equally valid) conv summation orders cannot flip a ReLU whose input is ~1e-7 from 0
    x = x + 1e-3 * np.random.default_rng(0).standard_normal(x.shape).astype(np.float32)
    torch.set_default_dtype(torch.float64)
    try:
        _ensemble_vs_sequential(tmp_path, x, y, xte, T, deeper)
    finally:
        torch.set_default_dtype(torch.float32)


def _ensemble_vs_sequential(tmp_path, x, y, xte, T, deeper):
    from mifx.privacy.pate import ensemble

    cfg = deep_cnn.DeepCNNConfig(max_steps=3, batch_size=16, nb_teachers=T, ckpt_every=2, deeper=deeper)
    shards = [deep_cnn.partition_dataset(x, y, T, t) for t in range(T)]
    seq = [str(tmp_path / f"seq{t}.ckpt") for t in range(T)]
    ens = [str(tmp_path / f"ens{t}.ckpt") for t in range(T)]
    for t in range(T):
        deep_cnn.train(shards[t][0], shards[t][1], seq[t], cfg, device="cpu", log=lambda *_: None)
    ensemble.train_ensemble([s[0] for s in shards], [s[1] for s in shards], ens, cfg, device="cpu",
                            log=lambda *_: None)
    for t in range(T):
        for step in (0, 2):
            a = torch.load(f"{seq[t]}-{step}", weights_only=True)
            b = torch.load(f"{ens[t]}-{step}", weights_only=True)
            assert a["step"] == b["step"] == step
            _states_close(a["state_dict"], b["state_dict"])
            _states_close(a["ema"], b["ema"])
    pe = ensemble.ensemble_softmax_preds(xte, [f"{p}-2" for p in ens], cfg, device="cpu")
    for t in range(T):
        ps = deep_cnn.softmax_preds(xte, f"{seq[t]}-2", cfg, device="cpu")
        np.testing.assert_allclose(pe[t], ps, rtol=1e-4, atol=1e-5)


def test_all_teachers_cli_and_student(tmp_path):
    common = ["--dataset", "mnist", "--train_dir", str(tmp_path), "--train_size", "900", "--test_size", "400",
              "--max_steps", "40", "--device", "cpu", "--batch_size", "64"]
    precisions = train_teachers.main(common + ["--nb_teachers", "3", "--teacher_id", "-1"])
    assert len(precisions) == 3 and min(precisions) > 0.5
    acc = train_student.main(common + ["--nb_teachers", "3", "--teachers_dir", str(tmp_path), "--data_dir",
                                       str(tmp_path), "--teachers_max_steps", "40", "--stdnt_share", "200",
                                       "--lap_scale", "0"])
    assert acc > 0.5


@pytest.mark.gpu
@pytest.mark.parametrize("deeper", [False, True])
@pytest.mark.parametrize("hip_conv", [False, True])
def test_ensemble_gpu_grads_match_per_teacher_models(monkeypatch, hip_conv, deeper):
    """On the GPU (grouped convs, HIP LRN kernel on per-teacher channel blocks, batched dense layers) the ensemble's
    fp32 logits and gradients equal each teacher's own PateCNN. With the hand-written bf16 grouped MFMA conv
    (csrc/gconv.hip, checked against fp32 in tests/test_gconv.py) the logits agree to bf16 accuracy."""
    import torch.nn.functional as F

    from mifx.privacy.pate import ensemble

    monkeypatch.setattr(ensemble, "USE_HIP_CONV", hip_conv)
    T, B = 5, 16
    cfg = deep_cnn.DeepCNNConfig(nb_teachers=T, deeper=deeper)
    torch.manual_seed(0)
    m = deep_cnn.build_model(cfg).cuda().to(memory_format=torch.channels_last)
    ens = ensemble.PateEnsemble(deep_cnn.build_model(cfg), T).cuda()
    states = []
    for t in range(T):  # distinct teachers
        st = {k: v + 0.01 * torch.randn_like(v) for k, v in m.state_dict().items()}
        states.append(st)
    ens.load_teachers(states)
    xs = [np.random.default_rng(t).random((B, 28, 28, 1)).astype(np.float32) for t in range(T)]
    ys = torch.randint(0, 10, (T, B), device="cuda")
    lo = ens(ensemble._interleave(xs, torch.device("cuda")))
    F.cross_entropy(lo.reshape(T * B, -1), ys.reshape(-1), reduction="sum").backward()
    grads = [p.grad for p in ens.parameters()]
    for t in range(T):
        m.load_state_dict(states[t])
        m.zero_grad()
        out = m(deep_cnn._to_nchw(xs[t], torch.device("cuda")))
        sc = out.abs().max()
        torch.testing.assert_close(lo[t].float() / sc, out / sc, rtol=0, atol=2e-2 if hip_conv else 1e-4)
        if hip_conv or deeper:  # deeper: 7 ReLU layers in fp32 -- gradient parity is the CPU fp64 test's job
            continue
        F.cross_entropy(out, ys[t], reduction="sum").backward()
        gt = ens.teacher_state(t, grads)
        for k, p in m.named_parameters():
            scale = p.grad.abs().max().clamp_min(1e-6)
            torch.testing.assert_close(gt[k] / scale, p.grad / scale, rtol=0, atol=2e-3, msg=k)


@pytest.mark.gpu
def test_ensemble_gpu_training_learns(tmp_path):
    from mifx.privacy.pate import ensemble

    T = 4
    x, y, xte, yte = deep_cnn.load_dataset("mnist", train_size=T * 512, test_size=256)
    shards = [deep_cnn.partition_dataset(x, y, T, t) for t in range(T)]
    cfg = deep_cnn.DeepCNNConfig(max_steps=60, batch_size=64, nb_teachers=T, ckpt_every=1000)
    ck = [str(tmp_path / f"t{t}.ckpt") for t in range(T)]
    ensemble.train_ensemble([s[0] for s in shards], [s[1] for s in shards], ck, cfg, device="cuda",
                            log=lambda *_: None)
    preds = ensemble.ensemble_softmax_preds(xte, [f"{c}-59" for c in ck], cfg, device="cuda")
    assert preds.shape == (T, 256, 10)
    assert min(float((p.argmax(1) == yte).mean()) for p in preds) > 0.5


def test_all_teachers_split_across_ranks(tmp_path, monkeypatch):
    """Under a multi-process launch rank r trains teachers r, r + W, ... and writes exactly their checkpoints."""
    common = ["--dataset", "mnist", "--train_dir", str(tmp_path), "--train_size", "400", "--test_size", "64",
              "--max_steps", "3", "--device", "cpu", "--batch_size", "32"]
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("WORLD_SIZE", "2")
    precisions = train_teachers.main(common + ["--nb_teachers", "4", "--teacher_id", "-1"])
    assert len(precisions) == 2
    names = sorted(p.name for p in tmp_path.glob("mnist_4_teachers_*.ckpt-2"))
    assert names == ["mnist_4_teachers_1.ckpt-2", "mnist_4_teachers_3.ckpt-2"]
