"""BERT flat-AdamW + hipGraph: back-to-back replays (bert_trainer.main's timing loop) vs synced replays,
with the default SDPA backend and with the math backend, and with dropout on/off. Prints the final
loss and whether parameters stayed finite, plus the first replay index whose loss is non-finite."""
import contextlib
import sys

import torch
from torch.nn.attention import SDPBackend, sdpa_kernel

sys.path.insert(0, ".")
from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402


def run(sync: bool, backend, dropout: float, steps: int = 40):
    torch.manual_seed(0)
    ctx = sdpa_kernel(backend) if backend is not None else contextlib.nullcontext()
    with ctx:
        cfg = BertConfig()
        cfg.dropout = dropout
        tr = BertTrainer(cfg, 32, 128, "cuda", graph=True, flat_adamw=True)
        hist = []
        for i in range(steps):
            loss = tr.step()
            if sync:
                hist.append(float(loss))
            else:
                hist.append(loss.clone())
        torch.cuda.synchronize()
    vals = [float(v) for v in hist]
    first_bad = next((i for i, v in enumerate(vals) if v != v or abs(v) == float("inf")), None)
    fin = all(torch.isfinite(p.float()).all().item() for p in tr.model.parameters())
    print(f"sync={sync} backend={backend} dropout={dropout}: final {vals[-1]:.4f} first_nonfinite={first_bad} "
          f"params_finite={fin} master_finite={bool(torch.isfinite(tr.opt.master).all())} "
          f"last5={[round(v, 4) for v in vals[-5:]]}", flush=True)


def main():
    print("BertConfig fields:", {k: v for k, v in vars(BertConfig()).items() if "drop" in k}, flush=True)
    run(False, None, 0.1)
    run(True, None, 0.1)
    run(False, None, 0.0)
    run(False, SDPBackend.MATH, 0.1)


if __name__ == "__main__":
    main()
