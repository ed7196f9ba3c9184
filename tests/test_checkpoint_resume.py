"""Estimator checkpoint / resume (reference RunConfig(save_checkpoints_steps=999, keep_checkpoint_max=1) and
warm_start_from, `airflow-dags/taxi_utils.py:333-336,345`): training N steps, checkpointing, and resuming to 2N
in a new estimator must equal an uninterrupted 2N run -- weights AND optimizer slots (Adagrad / FTRL
accumulators) restored -- bit-exact on the GPU's fused trainer, allclose on the CPU path."""
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from mifx.data.synthetic import synthetic_records
from mifx.trainer.estimator import RunConfig, WideDeepEstimator


def _est(d, device, warm=None, every=30):
    return WideDeepEstimator(RunConfig(model_dir=str(d), save_checkpoints_steps=every, keep_checkpoint_max=1,
                                       device=device), warm_start_from=warm, batch_size=64, steps_per_graph=7)


def _weights(est):
    return {k: v.detach().cpu().clone() for k, v in est.model.state_dict().items()}


def _resume_case(tmp_path, device, exact):
    recs = synthetic_records(64 * 50, seed=3)
    inp = lambda: recs.to(device)  # noqa: E731
    full = _est(tmp_path / "full", device).train(inp, 60)
    a = _est(tmp_path / "part", device).train(inp, 30)
    assert os.listdir(tmp_path / "part") == ["ckpt-30.safetensors"]
    b = _est(tmp_path / "part", device)  # restores ckpt-30: weights, optimizer slots, global step
    assert b.global_step == 30 and set(b._opt_state) == {"s0", "s1"}
    b.train(inp, 60)
    assert b.global_step == 60 and os.listdir(tmp_path / "part") == ["ckpt-60.safetensors"]
    wf, wb = _weights(full), _weights(b)
    for k in wf:
        if exact:
            assert torch.equal(wf[k], wb[k]), k
        else:
            np.testing.assert_allclose(wb[k].numpy(), wf[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
    sf = load_file(str(tmp_path / "full" / "ckpt-60.safetensors"))
    sb = load_file(str(tmp_path / "part" / "ckpt-60.safetensors"))
    for k in ("opt.s0", "opt.s1"):
        if exact:
            assert torch.equal(sf[k], sb[k]), k
        else:
            np.testing.assert_allclose(sb[k].numpy(), sf[k].numpy(), rtol=1e-5, atol=1e-6, err_msg=k)
    return a


def test_resume_equals_uninterrupted_cpu(tmp_path):
    _resume_case(tmp_path, "cpu", exact=False)


def test_warm_start_from_loads_weights(tmp_path):
    recs = synthetic_records(64 * 20, seed=4)
    a = _est(tmp_path / "a", "cpu").train(lambda: recs, 20)
    w = WideDeepEstimator(RunConfig(model_dir=str(tmp_path / "b"), device="cpu"), warm_start_from=str(tmp_path / "a"))
    assert w.global_step == 0  # warm start: weights only, a fresh run
    for k, v in _weights(a).items():
        assert torch.equal(w.model.state_dict()[k], v), k
    fresh = WideDeepEstimator(RunConfig(model_dir=str(tmp_path / "c"), device="cpu"))
    assert not all(torch.equal(fresh.model.state_dict()[k], v) for k, v in _weights(a).items())


def test_checkpoint_slots_are_trainer_independent(tmp_path):
    """The CPU trainer writes the fused trainer's canonical slot layout: Adagrad accumulators start at 0.1 and only
    grow; FTRL's linear slot moves."""
    recs = synthetic_records(64 * 20, seed=5)
    _est(tmp_path / "a", "cpu").train(lambda: recs, 20)
    sd = load_file(str(tmp_path / "a" / "ckpt-20.safetensors"))
    from mifx.models import wide_deep as wdm

    s0, s1 = sd["opt.s0"].numpy(), sd["opt.s1"].numpy()
    assert s0.shape == (wdm.WTOT + wdm.NWIDE,)
    assert (s0[wdm.WTOT:wdm.WTOT + 2127] >= 0.1 - 1e-7).all() and (s0[wdm.WTOT:] > 0.1).any()
    assert np.abs(s1[wdm.WTOT:]).max() > 0


@pytest.mark.gpu
def test_resume_equals_uninterrupted_gpu_bit_exact(tmp_path):
    """Fused trainer with multi-step hipGraph replays between checkpoints: bit-identical to the uninterrupted run."""
    _resume_case(tmp_path, "cuda", exact=True)
