"""Find where a BERT training variant goes non-finite (flat bf16 AdamW / hipGraph combinations)."""
import sys
import os

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402


def probe(flat, graph, layers=12, steps=8):
    tr = BertTrainer(BertConfig(layers=layers), 32, 128, "cuda", graph=graph, flat_adamw=flat)
    out = []
    for i in range(steps):
        out.append(round(float(tr.step()), 4))
    msg = f"flat={flat} graph={graph}: losses {out}"
    if flat:
        g = tr.opt.flat_grad.float()
        msg += f" | grad finite {bool(torch.isfinite(g).all())} max {float(g.abs().max()):.3g}"
        msg += f" | master finite {bool(torch.isfinite(tr.opt.master).all())}"
        bad = [n for n, p in tr.model.named_parameters() if not torch.isfinite(p.float()).all()]
        msg += f" | nonfinite params {bad[:5]}"
    print(msg, flush=True)


if __name__ == "__main__":
    for flat, graph in ((False, False), (True, False), (False, True), (True, True)):
        probe(flat, graph)
    # one eager flat step in detail: where do non-finite activations/grads appear?
    tr = BertTrainer(BertConfig(layers=12), 32, 128, "cuda", graph=False, flat_adamw=True)
    ids, tt, am, y = tr.data
    acts = {}

    def hook(name):
        def f(m, i, o):
            t = o[0] if isinstance(o, tuple) else o
            if torch.is_tensor(t) and name not in acts and not torch.isfinite(t.float()).all():
                acts[name] = True
        return f

    for n, m in tr.model.named_modules():
        m.register_forward_hook(hook(n))
    tr.opt.zero_grad()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        logits = tr.model(ids, tt, am)
    print("nonfinite forward modules (first few):", list(acts)[:8], flush=True)
    loss = F.cross_entropy(logits.float(), y)
    loss.backward()
    bad = [n for n, p in tr.model.named_parameters() if p.grad is not None and not torch.isfinite(p.grad.float()).all()]
    print("loss", float(loss), "nonfinite grads:", bad[:8], flush=True)
    print("grad views intact:", all(p.grad.data_ptr() >= tr.opt.flat_grad.data_ptr() and
                                    p.grad.data_ptr() < tr.opt.flat_grad.data_ptr() + tr.opt.flat_grad.numel() * 2
                                    for p in tr.model.parameters()), flush=True)
