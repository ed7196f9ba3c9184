"""Which aten ops (outside the hand-written kernels) an eager ResNet-50 B=256 training step launches: one profiled
step after warmup, torch.profiler; each aten op's count with its input shapes and self CUDA time, largest first."""
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet  # noqa: E402


def main():
    dev = torch.device("cuda")
    imgs, labels = synthetic_imagenet(512, seed=0, device=dev)
    tr = ResNetTrainer(256, dev, imgs, labels, warmup_steps=10, graph=False)
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA],
                                record_shapes=True) as prof:
        tr.step()
        torch.cuda.synchronize()
    rows = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.key_averages(group_by_input_shape=True):
        if ev.key.startswith("aten::") and ev.self_device_time_total > 0:
            r = rows[(ev.key, str(ev.input_shapes)[:140])]
            r[0] += ev.count
            r[1] += ev.self_device_time_total
    for (k, shp), (n, us) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{us:9.1f} us  {n:4d}x  {k:32s} {shp}")


if __name__ == "__main__":
    main()
