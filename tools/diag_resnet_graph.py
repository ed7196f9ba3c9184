"""ResNetTrainer losses, eager vs captured-graph steps, with and without a checkpoint restore in the middle
(the case tests/test_parallel_gpu.py::test_resnet_captured_step_matches_eager checks)."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet  # noqa: E402

imgs, labels = synthetic_imagenet(48, size=72, classes=10, seed=1)


def run(graph, restore_at=None, steps=7):
    tr = ResNetTrainer(6, "cuda:0", imgs, labels, num_classes=10, lr=0.05, warmup_steps=4, crop=64, seed=5,
                       graph=graph, graph_warmup=2)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    out = []
    with tempfile.TemporaryDirectory() as d:
        for i in range(steps):
            if restore_at is not None and i == restore_at:
                tr.restore(tr.save_checkpoint(d))
            out.append(round(float(tr.step()), 5))
    return out


for g, r in ((False, None), (False, 4), (True, None), (True, 4)):
    print(json.dumps({"graph": g, "restore_at": r, "losses": run(g, r)}), flush=True)
