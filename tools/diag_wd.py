"""Per-layer gradient diagnostics of the fused W&D kernel vs the bf16 emulation (GPU)."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models import wide_deep as wdm  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402
from tests.test_wide_deep import _emulated_grads  # noqa: E402

for batch in (40, 1000):
    m = wdm.WideDeepModel(seed=1)
    with torch.no_grad():
        m.wide.normal_(0, 0.3)
        for lin in m.dnn:
            lin.bias.normal_(0, 0.1)
    rec = synthetic_records(batch, seed=7)
    tr = FusedWideDeepTrainer(m, batch=batch, device="cuda")
    tr.set_data(rec.cuda())
    g = tr.gradients_once()
    gidx, mask = wdm.canonical_index_maps()
    got = g[gidx]
    _, em = _emulated_grads(tr.param.cpu(), rec)
    bounds = wdm.LAYER_OFF + [wdm.WTOT, wdm.WTOT + wdm.NWIDE]
    for li in range(6):
        s, e = bounds[li], bounds[li + 1]
        mk = mask[s:e].astype(bool)
        a, b = got[s:e][mk], em[s:e][mk]
        err = np.abs(a - b)
        print(f"B={batch} seg{li}: maxabs(em)={np.abs(b).max():.4g} maxerr={err.max():.4g} "
              f"relfro={np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-9):.4g}")
        if li < 5:
            K, N = wdm.LAYER_KN[li]
            ea = np.abs(got[s:e] - em[s:e]).reshape(N, K) * mask[s:e].reshape(N, K)
            n, k = np.unravel_index(np.argmax(ea), ea.shape)
            print(f"    worst at n={n} k={k}: got={got[s:e].reshape(N, K)[n, k]:.5g} em={em[s:e].reshape(N, K)[n, k]:.5g}")
