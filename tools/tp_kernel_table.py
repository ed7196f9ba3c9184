"""Kernel table of the tensor-parallel BERT step (ranks sharing one GPU: functional rehearsal of the TP path).

Spawns `--tp` ranks on cuda:0 (gloo for setup, the peer-memory all-reduce of mifx.parallel.tp_ipc for the TP
collectives), builds BertTrainer at that TP degree, and on rank 0 records `--active` eager steps with torch.profiler
(kernel names and GPU time per step), then times captured-graph steps. With every rank on ONE GPU the ranks' kernels
share its CUs, so per-kernel times are inflated by the other ranks' work; what the table shows is WHICH kernels a TP
step runs (the tpar_* all-reduce kernels in place of host collectives) and their relative cost.

    python tools/tp_kernel_table.py --tp 2 --layers 12 > profiles/bert_tp2_kernels_r4.md
"""
import argparse
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, a, out):
    from mifx.models.bert import BertConfig
    from mifx.parallel.tensor_parallel import TPGroup
    from mifx.trainer.bert_trainer import BertTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        lines = []
        for graph in (False, True):
            tp = TPGroup()
            torch.manual_seed(0)
            tr = BertTrainer(BertConfig(layers=a.layers), a.batch, a.seq, dev, tp, graph=graph, tp_ipc=True)
            for i in range(a.warmup):
                t0 = time.perf_counter()
                tr.step()
                if a.debug:  # host-synchronised warm-up steps with the group's health flag
                    torch.cuda.synchronize(dev)
                    print(f"[rank {rank}] graph={graph} warm-up step {i}: {time.perf_counter() - t0:.2f} s, "
                          f"err={int(tp.ipc.err.item()) if tp.ipc is not None else 0}", file=sys.stderr, flush=True)
            torch.cuda.synchronize(dev)
            prof = None
            if not graph and rank == 0 and not a.no_profile:  # (started before the barrier: the peers' kernels must not wait on rank 0
                # while it initialises the tracer -- the peer-memory waits time out after 10 s)
                from torch.profiler import ProfilerActivity, profile

                prof = profile(activities=[ProfilerActivity.CUDA])
                prof.__enter__()
            dist.barrier()
            if prof is not None:
                for _ in range(a.active):
                    tr.step()
                torch.cuda.synchronize(dev)
                prof.__exit__(None, None, None)
                rows = []
                for e in prof.key_averages():
                    t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
                    if t > 0:
                        rows.append((t, e.count, e.key))
                rows.sort(reverse=True)
                total = sum(r[0] for r in rows)
                ov = overlap_summary(prof)
                lines += [f"# TP={world} BERT step kernels (rank 0, eager, {a.active} steps; ranks share one GPU)", "",
                          f"batch {a.batch} seq {a.seq} layers {a.layers}; rank-0 GPU time per step "
                          f"{total / a.active / 1e3:.2f} ms", "",
                          "| kernel | calls/step | µs/step | % |", "|---|---|---|---|"]
                for t, c, k in rows[:a.top]:
                    lines.append(f"| `{k[:100]}` | {c / a.active:g} | {t / a.active:.1f} | {100 * t / total:.1f} |")
                lines += ["", "Streams (rank 0): " + ov]
            elif not graph:
                for _ in range(a.active):
                    tr.step()
                torch.cuda.synchronize(dev)
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                tr.step()
            torch.cuda.synchronize(dev)
            dt = (time.perf_counter() - t0) / a.steps
            dist.barrier()
            tp.check()
            if rank == 0:
                lines.append("")
                lines.append(f"{'captured hipGraph' if graph else 'eager'} step: {dt * 1e3:.2f} ms "
                             f"({a.steps} steps, all {world} ranks on one GPU)")
            tp.disable_ipc()
            del tr
        if rank == 0:
            with open(out, "w") as f:
                f.write("\n".join(lines) + "\n")
    finally:
        dist.destroy_process_group()


def overlap_summary(prof) -> str:
    """From the profiler's trace: kernels per GPU stream, and how much of the peer-memory all-reduce kernels' time
    (tpar_*) runs concurrently with a kernel on another stream (the row-parallel GEMM chunks, MIFX_TP_OVERLAP_CHUNKS)."""
    import json

    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "trace.json")
        prof.export_chrome_trace(path)
        ev = json.load(open(path)).get("traceEvents", [])
    ks = [e for e in ev if e.get("cat") == "kernel" and "dur" in e]
    if not ks:
        return "no kernel events in the trace"
    by_stream: dict = {}
    for e in ks:
        by_stream.setdefault(e.get("tid"), []).append(e)
    ar = [e for e in ks if e["name"].startswith(("tpar_", "void (anonymous namespace)::tpar", "(anonymous namespace)::tpar"))
          or "tpar_" in e["name"]]
    overlapped = 0.0
    for a in ar:
        a0, a1 = a["ts"], a["ts"] + a["dur"]
        cover = []
        for e in ks:
            if e.get("tid") == a.get("tid") or "tpar_" in e["name"]:
                continue
            lo, hi = max(a0, e["ts"]), min(a1, e["ts"] + e["dur"])
            if hi > lo:
                cover.append((lo, hi))
        cover.sort()
        t, end = 0.0, a0
        for lo, hi in cover:
            lo = max(lo, end)
            if hi > lo:
                t += hi - lo
                end = hi
        overlapped += t
    tot = sum(a["dur"] for a in ar)
    streams = ", ".join(f"stream {k}: {len(v)} kernels" for k, v in sorted(by_stream.items(), key=lambda kv: str(kv[0])))
    return (f"{streams}; all-reduce kernels {len(ar)}, {tot:.0f} us in total, {overlapped:.0f} us of it "
            f"({100 * overlapped / max(tot, 1e-9):.0f} %) concurrent with kernels on another stream")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=2)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--active", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--no-profile", action="store_true", help="step times only (no torch.profiler on rank 0)")
    ap.add_argument("--debug", action="store_true", help="per-rank warm-up step times and the all-reduce error flag")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "table.md")
        mp.start_processes(worker, args=(a.tp, _port(), a, out), nprocs=a.tp, start_method="spawn")
        print(open(out).read())


if __name__ == "__main__":
    main()
