"""Reproduce bert_trainer.main exactly, then inspect the trainer it used."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

import mifx.trainer.bert_trainer as bt  # noqa: E402

captured = {}
_orig = bt.BertTrainer.__init__


def _init(self, *a, **k):
    _orig(self, *a, **k)
    captured["tr"] = self


bt.BertTrainer.__init__ = _init

if __name__ == "__main__":
    bt.main(["--batch", "32", "--seq", "128", "--steps", "30", "--warmup", "5"])
    tr = captured["tr"]
    torch.cuda.synchronize()
    print("static loss", float(tr.static_loss) if tr.static_loss is not None else None)
    bad = [n for n, p in tr.model.named_parameters() if not torch.isfinite(p.float()).all()]
    print("nonfinite params:", bad[:10])
    if tr.flat:
        print("master finite", bool(torch.isfinite(tr.opt.master).all()), "m finite", bool(torch.isfinite(tr.opt.m).all()),
              "v finite", bool(torch.isfinite(tr.opt.v).all()), "grad finite", bool(torch.isfinite(tr.opt.flat_grad.float()).all()),
              "step", int(tr.opt.step_count))
    for i in range(5):
        print("extra step", i, float(tr.step()))
