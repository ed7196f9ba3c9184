"""Data-parallel engine on gloo, world_size 2 (CPU): bucketed/overlapped all-reduce must give the
same parameters as one process stepping on the concatenated global batch."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from mifx.data.synthetic import synthetic_records
from mifx.models import wide_deep as wdm
from mifx.parallel.ddp import DataParallel
from mifx.trainer.torch_wide_deep import TorchWideDeepTrainer


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _wd_worker(rank, world, port, out_dir, steps, batch):
    torch.manual_seed(0)
    _init(rank, world, port)
    recs = synthetic_records(batch * world * steps, device="cpu", seed=7)
    shard = recs.view(steps, world, batch, 32)[:, rank].reshape(-1, 32).contiguous()
    tr = TorchWideDeepTrainer(wdm.WideDeepModel(seed=3), batch=batch, process_group=dist.group.WORLD)
    tr.set_data(shard)
    for _ in range(steps):
        tr.step()
    if rank == 0:
        torch.save({k: v.detach().clone() for k, v in tr.model.state_dict().items()},
                   os.path.join(out_dir, "dp.pt"))
    dist.destroy_process_group()


def test_wide_deep_dp_matches_single_process():
    steps, batch, world = 3, 16, 2
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_wd_worker, args=(world, port, d, steps, batch), nprocs=world, start_method="spawn")
        got = torch.load(os.path.join(d, "dp.pt"), weights_only=True)
    torch.manual_seed(0)
    ref = TorchWideDeepTrainer(wdm.WideDeepModel(seed=3), batch=batch * world)
    recs = synthetic_records(batch * world * steps, device="cpu", seed=7)
    ref.set_data(recs)  # step i uses rows [i*2b, (i+1)*2b) == both ranks' shards of step i
    for _ in range(steps):
        ref.step()
    for k, v in ref.model.state_dict().items():
        np.testing.assert_allclose(got[k].numpy(), v.detach().numpy(), rtol=2e-5, atol=2e-6, err_msg=k)


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = torch.nn.Conv2d(1, 4, 3, padding=1)  # a 4-D weight: channels_last strides below
        self.a = torch.nn.Linear(16, 64)
        self.b = torch.nn.Linear(64, 64)
        self.unused = torch.nn.Linear(4, 4)
        self.c = torch.nn.Linear(64, 3)

    def forward(self, x):
        x = x + self.conv(x.view(-1, 1, 4, 4)).mean(1).reshape(-1, 16)
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))


def _ddp_worker(rank, world, port, out_dir, views=False):
    _init(rank, world, port)
    torch.manual_seed(100 + rank)  # different init per rank: DataParallel must broadcast rank 0's
    net = _Net().to(memory_format=torch.channels_last)
    dp = DataParallel(net, bucket_cap_mb=0.01, grad_as_bucket_view=views)  # tiny buckets -> several all-reduces
    assert len(dp.buckets) > 2
    if views:
        assert net.conv.weight.grad.stride() == net.conv.weight.stride()
        st = net.conv.weight.grad.untyped_storage().data_ptr()
        assert any(st == b.buf.untyped_storage().data_ptr() for b in dp.buckets)  # a view of a bucket
    g = torch.Generator().manual_seed(5)
    x = torch.randn(world * 8, 16, generator=g)
    y = torch.randint(0, 3, (world * 8,), generator=g)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    for _ in range(2):
        if views:
            dp.zero_grad()  # the bucket buffers are the gradients
        else:
            opt.zero_grad()
        with dp.no_sync():  # two micro-batches accumulated locally
            torch.nn.functional.cross_entropy(net(x[rank * 8:rank * 8 + 4]), y[rank * 8:rank * 8 + 4],
                                              reduction="sum").backward()
        torch.nn.functional.cross_entropy(net(x[rank * 8 + 4:rank * 8 + 8]), y[rank * 8 + 4:rank * 8 + 8],
                                          reduction="sum").backward()
        dp.finish()
        opt.step()
    if rank == 0:
        torch.save(net.state_dict(), os.path.join(out_dir, "ddp.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("views", [False, True])
def test_bucketed_ddp_matches_single_process(views):
    """Copy-in/copy-out buckets and gradients-as-bucket-views (no copies) give the single-process weights."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_ddp_worker, args=(world, port, d, views), nprocs=world, start_method="spawn")
        got = torch.load(os.path.join(d, "ddp.pt"), weights_only=True)
    torch.manual_seed(100)
    net = _Net()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(world * 8, 16, generator=g)
    y = torch.randint(0, 3, (world * 8,), generator=g)
    opt = torch.optim.SGD(net.parameters(), lr=0.1)
    for _ in range(2):
        opt.zero_grad()
        (torch.nn.functional.cross_entropy(net(x), y, reduction="sum") / world).backward()
        opt.step()
    for k, v in net.state_dict().items():
        np.testing.assert_allclose(got[k].numpy(), v.numpy(), rtol=1e-5, atol=1e-6, err_msg=k)


def _order_worker(rank, world, port, out_dir):
    _init(rank, world, port)
    torch.manual_seed(0)
    net = _Net()
    dp = DataParallel(net, bucket_cap_mb=0.01, grad_as_bucket_view=True, exchange="auto")
    assert dp.exchange == "rccl"  # CPU: no peer memory, the agreed fallback
    launched = []
    orig = dp._launch

    def rec(b, *a):
        launched.append(dp.buckets.index(b))
        orig(b, *a)

    dp._launch = rec
    params = [p for b in dp.buckets for p in b.params]
    order = list(range(len(params)))
    if rank == 1:
        order.reverse()  # the last bucket completes first on this rank
    for i in order:
        p = params[i]
        p.grad.fill_(float(rank + 1))
        dp._on_grad(p)
    dp.finish()
    ok = all(bool((p.grad == 1.5).all()) for p in params)  # (1 + 2) / 2
    torch.save({"launched": launched, "ok": ok, "n": len(dp.buckets)}, os.path.join(out_dir, f"order{rank}.pt"))
    dist.destroy_process_group()


def test_ddp_buckets_launch_in_order_whatever_completes_first():
    """Collectives must be issued in the same sequence on every rank: a bucket that completes before its
    predecessors waits for them (rank 1 completes the buckets in reverse)."""
    world, port = 2, _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_order_worker, args=(world, port, d), nprocs=world, start_method="spawn")
        r = [torch.load(os.path.join(d, f"order{k}.pt"), weights_only=True) for k in range(world)]
    for x in r:
        assert x["ok"] and x["launched"] == list(range(x["n"])), x


def test_ddp_ipc_exchange_needs_cuda():
    with pytest.raises(ValueError):
        DataParallel(_Net(), exchange="nope")


def test_ddp_coalesces_small_deferred_flushes(monkeypatch):
    """Buckets whose recorded products would not fill the GPU are not flushed alone: their flush (and exchange) waits
    until the run of complete buckets carries flush_min_wgs workgroups of work, else it is ONE flush in finish()."""
    from mifx.ops import gemm as hg

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(*[torch.nn.Linear(16, 16) for _ in range(4)])
        dp = DataParallel(net, bucket_cap_mb=0.0005, grad_as_bucket_view=True, force=True)
        assert len(dp.buckets) >= 4
        dp.deferred = True
        ws = [m.weight for m in net]
        pending = {id(w) for w in ws}
        calls, launches = [], []
        monkeypatch.setattr(hg, "pending_weights", lambda: set(pending))
        monkeypatch.setattr(hg, "pending_work", lambda weights: 300 * len(weights))

        def fake_flush(weights=None):
            calls.append(sorted(next(i for i, x in enumerate(ws) if x is w) for w in weights))
            for w in weights:
                pending.discard(id(w))
            return len(weights)

        monkeypatch.setattr(hg, "flush_weight_grads", fake_flush)
        launch = dp._launch
        dp._launch = lambda b, *a: (launches.append((any(any(p is w for w in ws) for p in b.params), len(calls))),
                                    launch(b, *a))
        dp.flush_min_wgs = 1024  # 4 weights' worth (300 each)
        dp.release_grads_for_defer()
        net(torch.randn(2, 16)).sum().backward()
        dp.finish()
        # backward completes the last layer's bucket first; 4 x 300 >= 1024 only with all four weights
        assert calls == [[0, 1, 2, 3]], calls
        # every bucket holding a deferred weight is exchanged after the one flush (bias-only buckets go at once)
        assert [n for has_w, n in launches if has_w] == [1, 1, 1, 1], launches
        assert len(launches) == len(dp.buckets)
    finally:
        dist.destroy_process_group()


def test_ddp_released_gradients_unused_parameter_gets_zero_slot():
    """release_grads_for_defer() replaces the per-step bucket memset: a parameter that receives no gradient in the step
    finds its (stale) bucket slot zeroed by finish() and its .grad re-attached as the view."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        net = torch.nn.ModuleDict({"a": torch.nn.Linear(4, 4), "unused": torch.nn.Linear(4, 4)})
        dp = DataParallel(net, grad_as_bucket_view=True, force=True)
        for b in dp.buckets:
            b.buf.fill_(5.0)  # stale contents from an earlier step
        dp.release_grads_for_defer()
        net["a"](torch.randn(3, 4)).sum().backward()
        dp.finish()
        for name, p in net.named_parameters():
            b, pi = dp._where[p]
            assert p.grad.data_ptr() == dp._view(dp.buckets[b], pi).data_ptr(), name
        assert torch.all(net["unused"].weight.grad == 0) and torch.all(net["unused"].bias.grad == 0)
        assert torch.all(net["a"].bias.grad == 3.0)
    finally:
        dist.destroy_process_group()


def test_ddp_deferred_flush_per_bucket_before_its_exchange(monkeypatch):
    """Deferred weight gradients under DataParallel: a bucket's recorded products are flushed (into its views) when the
    bucket's last gradient arrives, and its exchange is launched right after; a released 4-D weight whose gradient
    autograd produced itself is copied back into the bucket in the parameter's own (channels_last) layout."""
    from mifx.ops import gemm as hg

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.ReLU(), torch.nn.Conv2d(8, 8, 1),
                                  torch.nn.Flatten(), torch.nn.Linear(8 * 6 * 6, 4)).to(memory_format=torch.channels_last)
        dp = DataParallel(net, bucket_cap_mb=0.001, grad_as_bucket_view=True, force=True)
        assert len(dp.buckets) >= 3
        dp.deferred = True
        dp.flush_min_wgs = 0  # every complete bucket flushed at once (the coalescing threshold: next test)
        deferred_w = net[2].weight  # pretend the 1x1 conv's dW was recorded for a grouped flush
        events, pending = [], {id(deferred_w)}
        monkeypatch.setattr(hg, "pending_weights", lambda: set(pending))

        def fake_flush(weights=None):
            for w in weights:
                events.append(("flush", id(w)))
                w.grad.fill_(7.0)  # the product, written into the bucket view
                pending.discard(id(w))
            return len(weights)

        monkeypatch.setattr(hg, "flush_weight_grads", fake_flush)
        launch = dp._launch

        def spy(b, *a):
            events.append(("launch", next(i for i, q in enumerate(dp.buckets) if q is b)))
            launch(b, *a)

        dp._launch = spy
        dp.zero_grad()
        dp.release_grads_for_defer()
        assert all(p.grad is None for p in net.parameters())  # released: gradients are WRITTEN into the buckets
        x = torch.randn(2, 3, 8, 8).to(memory_format=torch.channels_last)

        class _Defer(torch.autograd.Function):  # what the conv ops do: a placeholder gradient, the product later
            @staticmethod
            def forward(ctx, w):
                return w.clone()

            @staticmethod
            def backward(ctx, g):
                return dp.grad_view(deferred_w)

        h = torch.relu(torch.nn.functional.conv2d(x, net[0].weight, net[0].bias))
        y = net[4](torch.nn.functional.conv2d(h, _Defer.apply(deferred_w), net[2].bias).flatten(1))
        y.square().sum().backward()
        dp.finish()
        bi = dp._where[deferred_w][0]
        assert events.index(("flush", id(deferred_w))) < events.index(("launch", bi)), events
        assert [e[1] for e in events if e[0] == "launch"] == list(range(len(dp.buckets)))
        assert torch.all(deferred_w.grad == 7.0)
        for p in net.parameters():  # every gradient IS its bucket view, in the parameter's layout
            b, pi = dp._where[p]
            v = dp._view(dp.buckets[b], pi)
            assert p.grad.data_ptr() == v.data_ptr() and p.grad.stride() == p.stride()
        assert net[0].weight.grad.abs().sum() > 0  # the released weight's own gradient, copied into its bucket
    finally:
        dist.destroy_process_group()


def test_ddp_check_forwards_the_exchange_error_and_guards_checkpoints(tmp_path):
    """DataParallel.check() raises the peer-memory exchange's sticky timeout, and ResNetTrainer refuses to write a
    checkpoint after one (the later buckets would be NaN)."""
    dp = DataParallel(_Net())
    dp.check()  # no exchange: nothing to report

    class FailedIpc:
        def check(self):
            raise RuntimeError("IPC all-reduce: a peer never published")

    dp._ipc = FailedIpc()
    with pytest.raises(RuntimeError, match="never published"):
        dp.check()
    from mifx.trainer.resnet_trainer import ResNetTrainer

    tr = ResNetTrainer.__new__(ResNetTrainer)
    tr.dp = dp
    with pytest.raises(RuntimeError, match="never published"):
        tr.save_checkpoint(str(tmp_path))
    assert not list(tmp_path.iterdir())


def test_tp_overlap_gate_needs_ipc_and_whole_chunks():
    """The overlapped row-parallel reduction applies only with the peer-memory all-reduce, TP > 1, token counts that
    split into whole 64-row chunks and chunks that fit the IPC buffer."""
    from mifx.parallel import tensor_parallel as tpm

    class FakeIpc:
        npad = 4096 * 768

    class FakeTP:
        size, ipc = 2, FakeIpc()

    saved = tpm._OVERLAP_CHUNKS
    try:
        tpm._OVERLAP_CHUNKS = 4
        assert tpm.overlap_ok(FakeTP(), 4096, 768)
        assert not tpm.overlap_ok(FakeTP(), 4096 + 64, 768)  # not whole 64-row chunks
        assert not tpm.overlap_ok(None, 4096, 768)
        t1 = FakeTP()
        t1.size = 1
        assert not tpm.overlap_ok(t1, 4096, 768)
        t2 = FakeTP()
        t2.ipc = None
        assert not tpm.overlap_ok(t2, 4096, 768)
        tpm._OVERLAP_CHUNKS = 1
        assert not tpm.overlap_ok(FakeTP(), 4096, 768)
        assert [sum(tpm.split_sizes(4096, 4, 64))] == [4096] and all(r % 64 == 0 for r in tpm.split_sizes(4096, 4, 64))
    finally:
        tpm._OVERLAP_CHUNKS = saved
