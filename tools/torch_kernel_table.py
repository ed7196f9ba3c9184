"""Steady-state per-kernel GPU time of a training step via torch.profiler (kineto/roctracer).

Unlike a whole-run rocprofv3 trace, warmup steps (MIOpen find, autotuning, first-touch allocation)
are excluded: the profiler records only the `--active` steps after `--warmup`.

    python tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > table.md
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402


def make_step(model: str, batch: int, seq: int):
    dev = torch.device("cuda")
    if model == "resnet":
        from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

        imgs, labels = synthetic_imagenet(1024, device=dev)
        tr = ResNetTrainer(batch, dev, imgs, labels, warmup_steps=10, graph=False)  # same kernels, visible
        return tr.step
    if model == "bert":
        from mifx.models.bert import BertConfig
        from mifx.trainer.bert_trainer import BertTrainer

        return BertTrainer(BertConfig(), batch, seq, dev, graph=False).step  # same kernels as the graph, visible
    raise ValueError(model)


def report_sources(step, active: int, pats) -> None:
    """For every kernel whose name contains one of `pats`: the launching CPU op and its Python stack, with counts."""
    from collections import Counter

    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(active):
            step()
        torch.cuda.synchronize()
    hits = Counter()
    for ev in prof.events():
        for k in getattr(ev, "kernels", []) or []:
            name = getattr(k, "name", str(k))
            for p in pats:
                if p in name:
                    stack = [f for f in (ev.stack or []) if "mifx" in f or "tools/" in f][:6]
                    hits[(p, ev.name, " <- ".join(stack))] += 1
    print(f"# kernel sources over {active} steps")
    for (p, op, stack), n in hits.most_common():
        print(f"- [{p}] x{n / active:.1f}/step  op `{op}`  {stack}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--active", type=int, default=5)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--sources", default="", help="comma-separated kernel-name substrings: report the Python "
                    "stacks (and CPU ops) that launched them instead of the table")
    a = ap.parse_args()
    from mifx.utils.meter import heartbeat

    step = make_step(a.model, a.batch, a.seq)
    with heartbeat(f"{a.model} warmup"):  # first steps: MIOpen solver search can run for minutes on a fresh box
        for i in range(a.warmup):
            step()
            torch.cuda.synchronize()
            print(f"[{a.model}] warmup step {i + 1}/{a.warmup}", file=sys.stderr, flush=True)
    from torch.profiler import ProfilerActivity, profile

    if a.sources:
        return report_sources(step, a.active, [p for p in a.sources.split(",") if p])
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(a.active):
            step()
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages():
        t = getattr(e, "device_time_total", None) or getattr(e, "cuda_time_total", 0)
        if t > 0:
            rows.append((t, e.count, e.key))
    rows.sort(reverse=True)
    total = sum(r[0] for r in rows)
    print(f"# steady-state kernels: {a.model} batch {a.batch}, {a.active} steps after {a.warmup} warmup\n")
    print(f"GPU time per step: {total / a.active / 1e3:.2f} ms\n")
    print("| kernel | calls/step | µs/step | % |\n|---|---|---|---|")
    for t, n, k in rows[:a.top]:
        print(f"| `{k[:110]}` | {n / a.active:.1f} | {t / a.active:.1f} | {100 * t / total:.1f} |")


if __name__ == "__main__":
    main()
