"""KFP taxi DNN: CPU oracle semantics + HIP gather/sparse-Adagrad kernels vs the oracle."""
import numpy as np
import pytest
import torch

from mifx.models.taxi_dnn import TaxiDNN, TaxiDNNConfig
from mifx.trainer.taxi_dnn_trainer import TaxiDNNTrainer


def _data(n, cfg, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.stack([torch.randint(0, size, (n,), generator=g) for _, size in cfg.sparse], 1)
    ids[:, 0] = torch.randint(0, 5, (n,), generator=g)  # repeated rows inside a batch
    dense = torch.randn(n, len(cfg.dense), generator=g)
    w = torch.randn(cfg.sparse_rows, generator=g)
    logit = w[ids + torch.as_tensor(cfg.offsets)].sum(1) * 0.5 + dense[:, 0]
    y = (torch.rand(n, generator=g) < torch.sigmoid(logit)).float()
    return ids, dense, y


def test_input_width_matches_reference():
    cfg = TaxiDNNConfig()
    assert cfg.input_dim == 6170 and cfg.sparse_rows == 6167
    assert sum(p.numel() for p in TaxiDNN(cfg).parameters()) == 6170 * 1500 + 1500 + 1500 + 1


def test_gather_forward_equals_one_hot_matmul():
    cfg = TaxiDNNConfig(hidden=64)
    m = TaxiDNN(cfg, seed=1)
    ids, dense, _ = _data(16, cfg)
    x = torch.zeros(16, cfg.input_dim)
    x.scatter_(1, m.rows(ids), 1.0)
    x[:, cfg.sparse_rows:] = dense
    ref = torch.relu(x @ m.W1 + m.b1) @ m.w2 + m.b2
    torch.testing.assert_close(m(ids, dense), ref, rtol=1e-5, atol=1e-5)


def test_cpu_training_reduces_loss():
    cfg = TaxiDNNConfig(hidden=128)
    ids, dense, y = _data(4096, cfg)
    tr = TaxiDNNTrainer(TaxiDNN(cfg, seed=0), batch=256, lr=0.1)
    tr.set_data(ids, dense, y)
    first = None
    for i in range(60):
        tr.step()
        first = first or tr.last_loss()
    assert tr.last_loss() < first


@pytest.mark.gpu
def test_hip_step_matches_cpu_oracle():
    cfg = TaxiDNNConfig()  # full 6170 x 1500
    ids, dense, y = _data(32 * 6, cfg, seed=4)
    cpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=2), batch=32, lr=0.1, device="cpu")
    gpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=2), batch=32, lr=0.1, device="cuda")
    for tr in (cpu, gpu):
        tr.set_data(ids, dense, y)
    for _ in range(6):
        cpu.step()
        gpu.step()
        assert gpu.last_loss() == pytest.approx(cpu.last_loss(), rel=1e-4)
    for n in ("W1", "b1", "w2", "b2"):
        torch.testing.assert_close(getattr(gpu.model, n).detach().cpu(), getattr(cpu.model, n).detach(),
                                   rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gpu.predict_logits(ids, dense), cpu.predict_logits(ids, dense), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("batch,steps,spg", [(32, 23, 5), (1024, 7, 3)])
def test_hip_graph_run_matches_cpu_oracle(batch, steps, spg):
    """run(): one eager step, then multi-step hipGraph replays + single-step replays; the device step counter walks
    the resident records exactly as the host oracle does (wrap-around included), and heavily repeated rows (field 0
    takes 5 values) exercise the in-kernel row dedup of the sparse Adagrad."""
    cfg = TaxiDNNConfig()
    ids, dense, y = _data(batch * 3 + 17, cfg, seed=7)  # not a multiple of the batch: batches wrap around
    cpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=3), batch=batch, lr=0.1, device="cpu")
    gpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=3), batch=batch, lr=0.1, device="cuda", steps_per_graph=spg)
    for tr in (cpu, gpu):
        tr.set_data(ids, dense, y)
    cpu.run(steps)
    gpu.run(steps)
    assert gpu.graph_multi is not None and gpu.step_idx == steps and int(gpu.step_ctr.item()) == steps
    assert gpu.last_loss() == pytest.approx(cpu.last_loss(), rel=2e-4)
    for n in ("W1", "b1", "w2", "b2"):
        torch.testing.assert_close(getattr(gpu.model, n).detach().cpu(), getattr(cpu.model, n).detach(),
                                   rtol=2e-4, atol=2e-5)


@pytest.mark.gpu
def test_set_data_twice_recaptures_graphs():
    """set_data after graph replays must drop the captured graphs (they hold the old tensors' addresses and
    record count); training on the new data then matches the CPU oracle fed the same two data sets."""
    cfg = TaxiDNNConfig()
    a = _data(32 * 4 + 5, cfg, seed=11)
    b = _data(32 * 2 + 3, cfg, seed=12)
    cpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=5), batch=32, lr=0.1, device="cpu")
    gpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=5), batch=32, lr=0.1, device="cuda", steps_per_graph=3)
    for d in (a, b):
        for tr in (cpu, gpu):
            tr.set_data(*d)
            tr.run(8)
        assert gpu.graph is not None
    assert gpu.last_loss() == pytest.approx(cpu.last_loss(), rel=2e-4)
    for n in ("W1", "b1", "w2", "b2"):
        torch.testing.assert_close(getattr(gpu.model, n).detach().cpu(), getattr(cpu.model, n).detach(),
                                   rtol=2e-4, atol=2e-5)
