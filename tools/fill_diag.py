"""Which Python lines launch the small elementwise kernels (fills, adds, copies) of an eager ResNet-50 step: one
profiled step after warmup, torch.profiler with stacks; prints each aten op's count and its top call sites."""
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet  # noqa: E402

OPS = ("aten::fill_", "aten::zero_", "aten::zeros", "aten::zeros_like", "aten::add_", "aten::add", "aten::copy_",
       "aten::mul", "aten::to", "aten::_to_copy", "aten::sum")


def main():
    dev = torch.device("cuda")
    imgs, labels = synthetic_imagenet(512, seed=0, device=dev)
    tr = ResNetTrainer(256, dev, imgs, labels, warmup_steps=10, graph=False)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                with_stack=True, record_shapes=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    sites = collections.defaultdict(collections.Counter)
    for ev in prof.events():
        if ev.name in OPS:
            st = [f for f in (ev.stack or []) if "mifx" in f or "tools" in f][:3]
            sites[ev.name][(" <- ".join(st) or "(no python frame)") + f"  shapes={ev.input_shapes[:1]}"] += 1
    for op, c in sites.items():
        print(f"== {op}: {sum(c.values())}")
        for k, v in c.most_common(12):
            print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main()
