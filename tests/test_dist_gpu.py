"""Multi-rank fused W&D trainer on one GPU: 2 processes share cuda:0 over gloo (RCCL refuses two
ranks on one device), exercising the split-graph step (local grad graph -> all-reduce -> optimizer
graph) that the 8-GPU RCCL run uses. Must match one process stepping on the global batch."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_dir, steps, batch):
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    recs = synthetic_records(batch * world * steps, device="cpu", seed=11)
    shard = recs.view(steps, world, batch, 32)[:, rank].reshape(-1, 32).contiguous()
    tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device="cuda:0",
                              process_group=dist.group.WORLD)
    tr.set_data(shard.cuda())
    tr.step()  # eager step, then split-graph capture for the rest
    tr.capture(warmup=0)
    for _ in range(steps - 1):
        tr.step()
    torch.cuda.synchronize()
    if rank == 0:
        m = tr.sync_to_model()
        torch.save({k: v.detach().cpu() for k, v in m.state_dict().items()}, os.path.join(out_dir, "dp.pt"))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_fused_dp_two_ranks_matches_single():
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    steps, batch, world = 4, 256, 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), d, steps, batch), nprocs=world,
                           start_method="spawn")
        got = torch.load(os.path.join(d, "dp.pt"), weights_only=True)
    tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch * world, device="cuda:0")
    tr.set_data(synthetic_records(batch * world * steps, device="cpu", seed=11).cuda())
    for _ in range(steps):
        tr.step()
    ref = tr.sync_to_model().state_dict()
    for k, v in ref.items():
        np.testing.assert_allclose(got[k].numpy(), v.detach().cpu().numpy(), rtol=2e-3, atol=2e-5, err_msg=k)


@pytest.mark.gpu
def test_captured_rccl_allreduce_step_matches_split_phase():
    """bench.py --capture-collective captures the RCCL all-reduce inside the step's hipGraph at N>1. On one GPU (1-rank RCCL
    group, trainer forced onto its data-parallel path) the captured step must produce exactly the weights
    of the split-phase step (graph, eager all-reduce, graph)."""
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        recs = synthetic_records(1 << 16, device="cuda", seed=4)
        out = []
        for captured in (False, True):
            tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=2), batch=4096, device="cuda",
                                      process_group=dist.group.WORLD)
            tr.world = 2  # take the DP code path (reduce_full -> all-reduce -> optimizer) on one rank
            tr.set_data(recs)
            tr.capture(include_collective=captured, dp_mode="split")
            assert (tr.graph is not None) == captured and (tr._graphs is not None) != captured
            for _ in range(6):
                tr.step()
            torch.cuda.synchronize()
            out.append(tr.param.clone())
        assert torch.equal(out[0], out[1])
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_direct_rccl_dp_step_matches_split_phase():
    """The default multi-rank W&D path (eager launches + ncclAllReduce on the compute stream through torch's
    communicator, mifx.parallel.rccl_direct) must give exactly the weights of the split-phase graph path, on a
    1-rank RCCL group with the trainer forced onto its data-parallel code path."""
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.parallel.rccl_direct import DirectAllReduce
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        x = torch.arange(1000, device="cuda", dtype=torch.float32)
        ar = DirectAllReduce(x)
        ar()
        torch.cuda.synchronize()
        assert torch.equal(x, torch.arange(1000, device="cuda", dtype=torch.float32))  # sum over one rank
        recs = synthetic_records(1 << 16, device="cuda", seed=4)
        out = []
        for mode in ("split", "direct"):
            tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=2), batch=4096, device="cuda",
                                      process_group=dist.group.WORLD)
            tr.world = 2
            tr.set_data(recs)
            tr.capture(dp_mode=mode)
            assert (tr._fast is not None) == (mode == "direct")
            tr.run(6)
            torch.cuda.synchronize()
            assert tr.steps_done == 8
            out.append(tr.param.clone())
        assert torch.equal(out[0], out[1])
    finally:
        dist.destroy_process_group()


def _xgmi_worker(rank, world, port, out_dir, steps, batch, spg, fused_wait=False):
    if fused_wait:  # read once by the library (csrc/wide_deep.hip): set before it loads
        os.environ["MIFX_XGMI_FUSED_WAIT"] = "1"
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        recs = synthetic_records(batch * world * steps, device="cpu", seed=11)
        shard = recs.view(steps, world, batch, 32)[:, rank].reshape(-1, 32).contiguous().cuda()
        out = {}
        for mode in ("split", "xgmi"):
            tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device="cuda:0",
                                      process_group=dist.group.WORLD)
            tr.set_data(shard)
            tr.step()  # one step on the collective path first
            tr.capture(warmup=1, steps_per_graph=spg, dp_mode=mode)
            if mode == "xgmi":
                assert tr.dp_exchange == "xgmi" and tr.graph is not None and tr.graph_multi is not None
            tr.run(steps - 2)
            torch.cuda.synchronize()
            assert tr.steps_done == steps
            if mode == "xgmi":
                tr._xg.check()
                tr.disable_xgmi()
            out[mode] = tr.param.cpu()
        torch.save(out, os.path.join(out_dir, f"xgmi{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world,batch,fused_wait", [(2, 512, False), (4, 512, False), (2, 8192, False),
                                                    (2, 65536, False), (4, 65536, False), (2, 65536, True)])
def test_xgmi_dp_step_matches_split_phase(world, batch, fused_wait):
    """Data parallelism over the one-shot xGMI exchange (IPC-shared HBM partials + epoch flags, csrc/xgmi.hip,
    wd_xgmi_opt): `world` processes share cuda:0 (the IPC path is the same as across GPUs) and run the step in
    multi-step hipGraphs with no host collective. Every replica must hold bit-identical weights, equal to the
    split-phase DP path (graph, all-reduce, graph): bit-exact at 2 ranks (a + b has one order), to fp32 summation
    order at 4. Batch 8192 (grid 64) takes the XCD-local local sum (wd_reduce_xcd + publish), 512 the one-pass one.
    Every rank's waits run in one-wave workgroups (wd_xgmi_gather_opt) on both paths, so ranks sharing one GPU
    always make progress; fused_wait=True is the opt-in variant whose 256-thread level-2 workgroups wait.
    (Against one process on the global batch both DP paths drift after ~6 steps on this data: FTRL's L1
    threshold flips wide weights on last-bit differences -- tools/xgmi_probe.py.)"""
    steps = 8
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_xgmi_worker, args=(world, _free_port(), d, steps, batch, 3, fused_wait), nprocs=world,
                           start_method="spawn")
        got = [torch.load(os.path.join(d, f"xgmi{r}.pt"), weights_only=True) for r in range(world)]
    for g in got[1:]:
        assert torch.equal(g["xgmi"], got[0]["xgmi"])
    if world == 2 and batch < 8192:
        assert torch.equal(got[0]["xgmi"], got[0]["split"])
    else:  # 4 ranks / XCD-local local sums: same math, other fp32 association
        np.testing.assert_allclose(got[0]["xgmi"].numpy(), got[0]["split"].numpy(), rtol=1e-4, atol=2e-6)


def _xgmi_timeout_worker(rank, world, port, out_dir, batch):
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device="cuda:0",
                                  process_group=dist.group.WORLD)
        tr.set_data(synthetic_records(batch * 2, device="cuda:0", seed=3))
        tr.enable_xgmi()  # collective self-test: both ranks healthy so far
        res = {}
        if rank == 0:  # rank 1 never joins the step: rank 0's wait must time out and leave the weights alone
            p0, s0 = tr.param.clone(), tr.s0.clone()
            tr._step_impl()
            tr._step_impl()  # the sticky error: a second exchange step does nothing at once
            torch.cuda.synchronize()
            res["err"] = int(tr._xg.err.item())
            res["param_unchanged"] = bool(torch.equal(tr.param, p0) and torch.equal(tr.s0, s0))
            try:
                tr.last_loss()
                res["raised"] = False
            except RuntimeError:
                res["raised"] = True
        dist.barrier()
        tr.disable_xgmi()
        torch.save(res, os.path.join(out_dir, f"to{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [512, 65536])
def test_xgmi_timeout_sets_err_skips_update_and_raises(batch):
    """A peer that never publishes: the bounded wall-clock wait (10 s) sets the sticky err flag, the exchange
    kernels then skip the parameter update and the counter advance, and the trainer raises at its next host sync
    instead of training on garbage (one-pass path at 512, XCD-local path at 65536)."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_xgmi_timeout_worker, args=(2, _free_port(), d, batch), nprocs=2, start_method="spawn")
        r = torch.load(os.path.join(d, "to0.pt"), weights_only=True)
    assert r == {"err": 1, "param_unchanged": True, "raised": True}
