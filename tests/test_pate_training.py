"""PATE-2017 training flow: batching, whitening, EMA checkpoints, teachers -> noisy-max -> student."""
import math

import numpy as np
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
