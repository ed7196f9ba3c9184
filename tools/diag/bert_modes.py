"""BERT-base trainer loss trajectory in each optimizer / capture mode (finds which combination
produces a non-finite loss): torch fused AdamW vs flat HIP AdamW, eager vs hipGraph."""
import sys

import torch

sys.path.insert(0, ".")
from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    for flat, graph in ((False, False), (True, False), (False, True), (True, True)):
        tr = BertTrainer(BertConfig(layers=12), 32, 128, dev, graph=graph, flat_adamw=flat)
        losses = []
        for _ in range(10):
            losses.append(round(float(tr.step()), 4))
        torch.cuda.synchronize()
        bad = [n for n, p in tr.model.named_parameters() if not torch.isfinite(p.float()).all()]
        extra = ""
        if flat:
            extra = (f" master_finite={bool(torch.isfinite(tr.opt.master).all())}"
                     f" grad_finite={bool(torch.isfinite(tr.opt.flat_grad.float()).all())}"
                     f" step={int(tr.opt.step_count)}")
        print(f"flat={flat} graph={graph} losses={losses} nonfinite_params={bad[:4]}{extra}", flush=True)
        del tr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
