"""40-step losses: flat AdamW + hipGraph, and hipGraph + TunableOp-selected GEMMs."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402


def run(graph, flat, steps=40, tag=""):
    tr = BertTrainer(BertConfig(), 32, 128, "cuda", graph=graph, flat_adamw=flat)
    losses = [round(float(tr.step()), 4) for _ in range(steps)]
    first_bad = next((i for i, v in enumerate(losses) if v != v), None)
    print(f"{tag} graph={graph} flat={flat}: first NaN step {first_bad}; {losses}", flush=True)


if __name__ == "__main__":
    run(True, True, tag="plain")
    run(False, True, tag="plain")
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    torch.cuda.tunable.read_file("profiles/tunableop_bert_base_mi355x.csv")
    run(False, False, tag="tunable")
    run(True, False, tag="tunable")
