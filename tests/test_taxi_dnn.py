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


def _dp_worker(rank, world, port, out, device, batch, steps, hidden):
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = TaxiDNNConfig(hidden=hidden)
        ids, dense, y = _data(batch * world * steps + 7, cfg, seed=21)
        tr = TaxiDNNTrainer(TaxiDNN(cfg, seed=rank + 1), batch=batch, lr=0.1, device=device,  # rank 0's init wins
                            process_group=dist.group.WORLD)
        tr.set_data(ids, dense, y)
        tr.run(steps)
        torch.save({n: getattr(tr.model, n).detach().cpu() for n in ("W1", "b1", "w2", "b2")}, f"{out}.{rank}")
    finally:
        dist.destroy_process_group()


def _dp_case(tmp_path, device, batch, steps, hidden):
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "dp")
    mp.start_processes(_dp_worker, args=(2, port, out, device, batch, steps, hidden), nprocs=2, start_method="spawn")
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in (0, 1))
    cfg = TaxiDNNConfig(hidden=hidden)
    ids, dense, y = _data(batch * 2 * steps + 7, cfg, seed=21)
    n = batch * 2 * steps  # the DP shards drop the last partial global batch
    one = TaxiDNNTrainer(TaxiDNN(cfg, seed=1), batch=2 * batch, lr=0.1, device=device)
    one.set_data(ids[:n], dense[:n], y[:n])
    one.run(steps)
    ref = {k: getattr(one.model, k).detach().cpu() for k in ("W1", "b1", "w2", "b2")}
    return r0, r1, ref


def test_dp_cpu_two_ranks_equal_one_process_global_batch(tmp_path):
    r0, r1, ref = _dp_case(tmp_path, "cpu", 16, 6, 64)
    for k in ref:
        assert torch.equal(r0[k], r1[k]), k
        torch.testing.assert_close(r0[k], ref[k], rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [32, 48])
def test_dp_gpu_sparse_exchange_bit_identical_to_global_batch(tmp_path, batch):
    """Two ranks sharing cuda:0 exchange per-example backward state (one all-gather) and run the sparse + dense
    Adagrad kernels over the global batch: bit-identical to one process at batch 2B (2B = 64: per-example dense
    chunks travel too; 96: the chunked reduction path)."""
    r0, r1, ref = _dp_case(tmp_path, "cuda", batch, 5, 1500)
    for k in ref:
        assert torch.equal(r0[k], r1[k]), k
        assert torch.equal(r0[k], ref[k]), k
