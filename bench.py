#!/usr/bin/env python
"""Headline benchmark: Trainer examples/sec (whole node), Chicago-Taxi Wide&Deep, 1/2/4/8 MI355X.

Model: the reference W&D (`airflow-dags/taxi_utils.py:148-191,300-345`): DNN [100,70,48,34] on
3 dense floats + linear part over 9 categorical identity columns (2127 buckets), sigmoid CE,
Adagrad(DNN) + FTRL(linear) — full training step (fwd + bwd + all-reduce + optimizer) in the
timed region. Data: synthetic transformed-taxi records resident in HBM (no network for the
real CSV); random-init weights. Weak scaling: fixed batch per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch-per-gpu B]
    torchrun --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1, no torchrun env) starts its own N ranks -- one process per GPU with
torchrun-style env, spawned before this process touches the GPU -- relays rank 0's JSON line and exits with the
worst rank's code (a failing rank takes the job down), like the job-owned replicas of the reference's
`notebooks/training-jobs/distributed-tensorflow-training-job.yaml:8-18`. Under torchrun, WORLD_SIZE must equal
--gpus: a mismatch exits non-zero instead of timing a different number of GPUs than was asked for.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.parallel import dist as mdist  # noqa: E402

METRIC = "Trainer examples/sec (whole node), Chicago-Taxi Wide&Deep at 1/2/4/8 MI355X"
MODEL = "chicago-taxi-wide-deep (DNNLinearCombinedClassifier: dnn [100,70,48,34] on 3 dense, linear on 9 cat cols)"


def run(trainer, steps: int, warmup: int, device) -> float:
    for _ in range(warmup):
        trainer.step()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    mdist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    if hasattr(trainer, "run"):
        trainer.run(steps)  # exactly `steps` steps (multi-step graph replays + one-step remainder)
    else:
        for _ in range(steps):
            trainer.step()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    mdist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    return time.perf_counter() - t0


def _ranks_agree(tr) -> bool:
    """All ranks apply the same all-reduced gradient to the same initial weights: their parameters must be
    bit-identical. Eager MAX/MIN all-reduce of a checksum, outside any graph."""
    prm = tr.param if hasattr(tr, "param") else torch.cat([p.detach().flatten() for p in tr.model.parameters()])
    chk = torch.stack([prm.double().sum(), prm.double().abs().sum()])
    hi, lo = chk.clone(), chk.clone()
    torch.distributed.all_reduce(hi, op=torch.distributed.ReduceOp.MAX)
    torch.distributed.all_reduce(lo, op=torch.distributed.ReduceOp.MIN)
    return bool(torch.equal(hi, lo)) and bool(torch.isfinite(chk).all())


def _post_run_ok(tr, n: int, use_cuda: bool) -> tuple[bool, bool | None]:
    """After the timed region (outside it): the exchange must not have timed out on any rank and every replica
    must hold bit-identical weights. Returns (ok on every rank, replicas_bit_identical or None at one rank)."""
    if n == 1:
        return True, None
    if not use_cuda:
        agree = _ranks_agree(tr)
        return agree, agree
    bad = 0.0
    try:
        if getattr(tr, "_xg", None) is not None:
            tr._xg.check()
    except RuntimeError as e:
        print(f"[bench] {e}", file=sys.stderr, flush=True)
        bad = 1.0
    flag = torch.tensor([bad], device=tr.device)
    torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
    agree = _ranks_agree(tr)
    return flag.item() == 0.0 and agree, agree


def gradient_check(batch: int, device, seed: int) -> float:
    """Outside the timed region: ONE training step through the same kernels the benchmark times (fused fwd/bwd,
    XCD-local slab reduction, slab-order optimizer) with plain SGD at lr 1, so the weight change IS the summed
    gradient, against fp32 PyTorch autograd of the same model on the same records. Returns the largest relative
    Frobenius error over the parameter tensors: the bf16 data path costs a few % (tests/test_wide_deep.py); a
    broken reduction, exchange or optimizer shows up as O(1)."""
    import numpy as np

    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer, OptSpec

    recs = synthetic_records(batch, device=device, seed=seed)
    tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device=device, dnn_opt=OptSpec("sgd", lr=1.0),
                              wide_opt=OptSpec("sgd", lr=1.0))
    tr.set_data(recs)
    before = tr.param.double().cpu()
    tr.step()
    torch.cuda.synchronize(device)
    g = (before - tr.param.double().cpu()).float().numpy()
    got = wdm.canonical_grad_to_torch(g, tr.model, np.arange(g.size))
    ref_model = wdm.unpack_canonical(before.float(), WideDeepModel(seed=0))
    dense, ids, label = wdm.records_to_tensors(recs.cpu())
    ref_model.zero_grad()
    ref_model.loss(dense, ids, label, reduction="sum").backward()
    worst = 0.0
    for name, prm in ref_model.named_parameters():
        r = prm.grad.detach().numpy()
        gk = np.asarray(got[name]).reshape(r.shape)
        worst = max(worst, float(np.linalg.norm(gk - r) / (np.linalg.norm(r) + 1e-8)))
    del tr
    return worst


def make_trainer(batch: int, device, pg, seed: int, n_data: int, graph: bool, dp: str = "xgmi",
                 steps_per_graph: int = 10, shuffle_seed: int = 0):
    def build():
        model = WideDeepModel(seed=0)
        if device.type == "cuda":
            from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

            t = FusedWideDeepTrainer(model, batch=batch, device=device, process_group=pg, shuffle_seed=shuffle_seed)
        else:
            from mifx.trainer.torch_wide_deep import TorchWideDeepTrainer

            t = TorchWideDeepTrainer(model, batch=batch, device=device, process_group=pg, shuffle_seed=shuffle_seed)
            t.dp_path = "gloo bucketed all-reduce (mifx.parallel.ddp)" if pg is not None else None
        t.set_data(synthetic_records(n_data, device=device, seed=seed))
        return t

    tr = build()
    if not (graph and device.type == "cuda"):
        return tr
    if pg is None:
        tr.capture(steps_per_graph=steps_per_graph)
        tr.dp_path = None
        return tr
    # Multi-rank data parallelism, default "xgmi": the one-shot xGMI gradient exchange (mifx.parallel.xgmi) --
    # every rank reads its peers' 82 KB local gradients straight from their HBM and sums + applies the optimizer
    # in one kernel, device-side epoch flags keep the ranks in lock-step, so the whole step (and 10 of them) is
    # one hipGraph with no host collective. Guard: its setup self-test, then 2 graph replays after which every
    # rank must hold bit-identical weights with no timed-out wait; otherwise (agreed by all ranks) the trainer is
    # released and the "direct" path is built: eager launches + ncclAllReduce enqueued on the compute stream
    # through torch's RCCL communicator (mifx.parallel.rccl_direct). "captured" puts the RCCL all-reduce inside
    # the step's graph, "split" issues torch's all_reduce between two graphs.
    if dp == "xgmi":
        ok = True
        try:
            tr.capture(steps_per_graph=steps_per_graph, dp_mode="xgmi")
            tr.run(2 * max(1, steps_per_graph))
            torch.cuda.synchronize(device)
            tr._xg.check()
        except Exception as e:  # noqa: BLE001 -- agreed on below
            print(f"[bench] xGMI exchange unavailable: {e}", file=sys.stderr, flush=True)
            ok = False
        flag = torch.tensor([0.0 if ok else 1.0], device=device)
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MAX)
        ok = flag.item() == 0.0 and _ranks_agree(tr)
        if ok:
            tr.dp_path = "xgmi one-shot exchange (IPC peer reads + epoch flags, whole step in hipGraphs)"
            return tr
        print("[bench] xGMI step failed validation on some rank: falling back to direct RCCL", file=sys.stderr,
              flush=True)
        if tr._xg is not None:
            tr.disable_xgmi()
        del tr
        torch.cuda.synchronize(device)
        torch.cuda.empty_cache()
        tr = build()
        dp = "direct"
    captured = dp == "captured" and torch.distributed.get_backend(pg) == "nccl"
    tr.capture(include_collective=captured, steps_per_graph=steps_per_graph,
               dp_mode="split" if dp == "split" else "direct")
    tr.dp_path = ("captured-in-graph" if captured else
                  "rccl-direct (eager launches + ncclAllReduce on the compute stream)" if tr._fast is not None else
                  "split-phase graphs + torch all_reduce")
    if captured:
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize(device)
        if not _ranks_agree(tr):
            print("[bench] captured all-reduce: ranks disagree, falling back to split-phase graphs",
                  file=sys.stderr, flush=True)
            del tr
            torch.cuda.synchronize(device)
            torch.cuda.empty_cache()
            tr = build()
            tr.capture(dp_mode="split")
            tr.dp_path = "split-phase graphs + torch all_reduce"
    return tr


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Run this script as N ranks (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), one per
    GPU. Nothing here touches the GPU (no torch.cuda call): the native libraries are checked (and rebuilt if stale)
    once, under the build lock, before any rank starts. Rank 0's stdout is relayed line by line; every rank's
    stderr goes to ours. The first rank that fails kills the others and its exit code is the job's."""
    try:
        from mifx.ops import build

        build.build_all(verbose=False)
    except Exception as e:  # noqa: BLE001 -- no hipcc / read-only tree: the ranks' own load() reports it
        print(f"[bench] native prebuild skipped: {e}", file=sys.stderr, flush=True)
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0",
                   MIFX_AUTOBUILD="0")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, start_new_session=True))

    def relay():
        for line in procs[0].stdout:  # the result line to stdout; library chatter (gloo, RCCL) to stderr
            txt = line.decode()
            out = sys.stdout if txt.lstrip().startswith("{") else sys.stderr
            out.write(txt)
            out.flush()

    t = threading.Thread(target=relay, daemon=True)
    t.start()
    codes = [None] * n
    first_bad = None
    try:
        while any(c is None for c in codes):
            codes = [p.poll() for p in procs]
            if any(c not in (None, 0) for c in codes):
                bad = next(r for r, c in enumerate(codes) if c not in (None, 0))
                first_bad = codes[bad]
                print(f"[bench] rank {bad} exited with {codes[bad]}: stopping the job", file=sys.stderr, flush=True)
                break
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
            p.wait()
        t.join(timeout=5)
    codes = [(c if c >= 0 else 128 - c) for c in (p.returncode for p in procs)]  # signal death -> 128+sig
    if first_bad is not None:  # the rank that failed first is the cause; the ones killed after it are not
        return first_bad if first_bad >= 0 else 128 - first_bad
    return max(codes)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch-per-gpu", type=int, default=65536,
                    help="throughput batch per replica (BASELINE.md protocol: 8K-64K); 40 = reference batch")
    ap.add_argument("--ref-batch", type=int, default=40, help="also time the reference batch (0 = skip)")
    ap.add_argument("--ref-steps", type=int, default=2000)
    ap.add_argument("--ref-steps-per-graph", type=int, default=100,
                    help="steps per hipGraph for the reference-batch run (its 2000 steps amortise graph boundaries; "
                         "profiles/archive/bench_ref_spg_sweep_r3.txt)")
    ap.add_argument("--data-per-gpu", type=int, default=1 << 24, help="resident records per GPU (32 B each)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--shuffle-seed", type=int, default=0x5EED,
                    help="per-epoch shuffle of the resident records inside the kernel's record fetch (csrc/feed.h; "
                         "the reference's read_batch_features(randomize_input=True)); 0 = stored order")
    ap.add_argument("--steps-per-graph", type=int, default=20,
                    help="consecutive training steps captured in one hipGraph (single rank / captured collective); "
                         "20 measured best at the driver's 20 timed steps (profiles/archive/bench_spg_sweep_r3.txt)")
    ap.add_argument("--dp", choices=("xgmi", "direct", "captured", "split"), default="xgmi",
                    help="multi-rank gradient exchange: xgmi (one-shot peer reads, whole step in hipGraphs; falls "
                         "back to direct if its validation fails), direct (eager + ncclAllReduce on the compute "
                         "stream), captured (RCCL all-reduce inside the graph), split (torch all_reduce between "
                         "two graphs)")
    a = ap.parse_args(argv)

    ws = os.environ.get("WORLD_SIZE")
    if ws is None and a.gpus > 1:
        return spawn_ranks(a.gpus, argv)
    if int(ws or 1) != a.gpus:
        print(f"[bench] WORLD_SIZE={ws} but --gpus {a.gpus}: refusing to time a different number of GPUs",
              file=sys.stderr, flush=True)
        return 2
    env = mdist.init()
    if os.environ.get("MIFX_BENCH_FAIL_RANK") == str(env.rank):  # fault injection (tests): this rank dies
        print(f"[bench] rank {env.rank}: injected failure", file=sys.stderr, flush=True)
        os._exit(3)
    use_cuda = torch.cuda.is_available()
    # MIFX_SHARED_GPU=1 (rehearsal of the multi-rank flow on a 1-GPU box, with MIFX_DIST_BACKEND=gloo): every
    # rank on cuda:0 -- functional only, the timings of ranks sharing a GPU mean nothing
    shared = os.environ.get("MIFX_SHARED_GPU") == "1"
    device = torch.device("cuda", 0 if shared else env.local_rank) if use_cuda else torch.device("cpu")
    if use_cuda:
        torch.cuda.set_device(device)
    else:  # CPU dev fallback: keep it quick
        a.batch_per_gpu = min(a.batch_per_gpu, 4096)
        a.data_per_gpu = min(a.data_per_gpu, 1 << 16)
        a.steps, a.warmup, a.ref_steps = min(a.steps, 20), min(a.warmup, 2), min(a.ref_steps, 50)
    pg = torch.distributed.group.WORLD if env.world_size > 1 else None
    n = env.world_size
    seen = torch.distributed.get_world_size() if pg is not None else 1
    if seen != a.gpus:
        raise SystemExit(f"[bench] process group has {seen} ranks, --gpus {a.gpus}")

    def measure(batch, seed, n_data, steps, warmup, spg_req=None):
        """Build, time `steps` steps, validate after the timed region. A multi-rank xGMI run that fails the
        post-run validation (a timed-out wait, replicas that differ) is discarded and re-measured on the direct
        RCCL path; a failing direct run fails the benchmark (no number from a broken step)."""
        dp = a.dp
        while True:
            tr = make_trainer(batch, device, pg, seed, n_data, not a.no_graph, dp, spg_req or a.steps_per_graph,
                              a.shuffle_seed)
            spg = int(getattr(tr, "graph_multi_steps", 1)) if getattr(tr, "graph_multi", None) is not None else 1
            dt = mdist.max_over_ranks(run(tr, steps, warmup, device), device if use_cuda else None)
            ok, agree = _post_run_ok(tr, n, use_cuda)
            res = {"dt": dt, "dp_path": getattr(tr, "dp_path", None), "spg": spg, "agree": agree,
                   "loss": tr.last_loss() / batch if ok else float("nan")}
            if pg is not None:  # which exchange every rank actually timed
                paths = [None] * n
                torch.distributed.all_gather_object(paths, res["dp_path"])
                res["dp_per_rank"] = paths
            if getattr(tr, "_xg", None) is not None:
                tr.disable_xgmi()
            del tr
            if use_cuda:
                torch.cuda.synchronize(device)
                torch.cuda.empty_cache()
            if ok:
                return res
            if dp == "direct":
                raise SystemExit("[bench] the direct RCCL step failed post-run validation")
            print("[bench] post-run validation failed: re-measuring on the direct RCCL path", file=sys.stderr,
                  flush=True)
            dp = "direct"

    r = measure(a.batch_per_gpu, 1234 + env.rank, a.data_per_gpu, a.steps, a.warmup)
    dt, dp_path, spg, ranks_agree, loss = r["dt"], r["dp_path"], r["spg"], r["agree"], r["loss"]
    dp_per_rank = r.get("dp_per_rank")
    value = a.batch_per_gpu * n * a.steps / dt
    grad_err = None
    if use_cuda and env.is_main:  # after the timed region: the kernel's gradient vs fp32 autograd on one batch
        grad_err = gradient_check(a.batch_per_gpu, device, 4321)
        if not grad_err < 0.1:
            raise SystemExit(f"[bench] gradient check failed: relative error {grad_err:.3g} vs fp32 autograd")

    ref = None
    if a.ref_batch:
        r2 = measure(a.ref_batch, 99 + env.rank, 1 << 16, a.ref_steps, max(10, a.warmup),
                     min(a.ref_steps_per_graph, max(1, a.ref_steps)))
        ref = {"batch_per_gpu": a.ref_batch, "examples_per_sec": a.ref_batch * n * a.ref_steps / r2["dt"],
               "ms_per_step": 1e3 * r2["dt"] / a.ref_steps, "steps": a.ref_steps,
               "dp_exchange": r2["dp_path"], "dp_exchange_per_rank": r2.get("dp_per_rank"),
               "replicas_bit_identical": r2["agree"]}

    if env.is_main:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "examples/s",
            "n_gpus": n,
            "world_size_seen_by_backend": seen,
            "backend": torch.distributed.get_backend(pg) if pg is not None else None,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": 1e3 * dt / a.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if use_cuda else "fp32",
            "data": "synthetic (transformed Chicago-Taxi-shaped records, HBM-resident, "
                    + ("reshuffled every epoch in-kernel" if a.shuffle_seed else "stored order")
                    + "); random-init weights",
            "config": {"model": MODEL, "global_batch": a.batch_per_gpu * n, "seq_len": None,
                       "parallelism": f"dp{n}", "batch_per_gpu": a.batch_per_gpu,
                       "optimizer": "adagrad(dnn,lr=0.05)+ftrl(linear,lr=0.2)",
                       "precision": "bf16 MFMA compute, fp32 master weights/optimizer state",
                       "device": torch.cuda.get_device_name(device) if use_cuda else "cpu",
                       "hipgraph": bool(use_cuda and not a.no_graph),
                       "input_shuffle_seed": a.shuffle_seed,
                       "steps_per_graph": spg,
                       "kernel": "wd_chain (register-chained, 8 waves)" if use_cuda else "torch-cpu",
                       "dp_exchange": dp_path, "dp_exchange_per_rank": dp_per_rank,
                       "replicas_bit_identical": ranks_agree, "validated_after_timed_region": True,
                       "grad_check_max_rel_err_vs_fp32": grad_err},
            "final_mean_loss": loss,
            "reference_batch": ref,
        }
        print(json.dumps(out))
    mdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
