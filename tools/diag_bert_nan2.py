"""Per-step losses over 40 steps for eager / hipGraph BERT training (dropout 0.1 and 0.0)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402


def run(graph, flat, dropout, steps=40):
    tr = BertTrainer(BertConfig(dropout=dropout), 32, 128, "cuda", graph=graph, flat_adamw=flat)
    losses = [round(float(tr.step()), 4) for _ in range(steps)]
    first_bad = next((i for i, v in enumerate(losses) if v != v), None)
    print(f"graph={graph} flat={flat} dropout={dropout}: first NaN step {first_bad}; {losses}", flush=True)
    return tr, first_bad


if __name__ == "__main__":
    run(False, False, 0.1)
    run(True, False, 0.0)
    tr, bad = run(True, False, 0.1)
    run(False, True, 0.1)
