"""Does back-to-back hipGraph replay (no host sync between steps) go non-finite where synced replay
does not? Mirrors bert_trainer.main's timing loop."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.models.bert import BertConfig  # noqa: E402
from mifx.trainer.bert_trainer import BertTrainer  # noqa: E402

if __name__ == "__main__":
    for flat in (True, False):
        for sync_every in (0, 1):
            torch.manual_seed(0)
            tr = BertTrainer(BertConfig(), 32, 128, "cuda", graph=True, flat_adamw=flat)
            seen = []
            for i in range(40):
                loss = tr.step()
                if sync_every and i % sync_every == 0:
                    seen.append(round(float(loss), 4))
            torch.cuda.synchronize()
            print(f"flat={flat} sync_every={sync_every}: final {float(loss):.4f} "
                  f"finite-params {all(torch.isfinite(p.float()).all().item() for p in tr.model.parameters())} "
                  f"seen {seen[-5:]}", flush=True)
    # eager, no sync (the configuration whose bench loss was finite)
    tr = BertTrainer(BertConfig(), 32, 128, "cuda", graph=False, flat_adamw=True)
    for i in range(40):
        loss = tr.step()
    torch.cuda.synchronize()
    print(f"eager flat no-sync: final {float(loss):.4f}", flush=True)
