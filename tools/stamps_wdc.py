"""Phase breakdown of wdc_fused<true> (csrc/wd_chain.hip) block 0 via the s_memtime diagnostic build.

Build: bash tools/build_stamps.sh (CPU) -> tools/bin/libwdc_stamps.so; run on the GPU: python tools/stamps_wdc.py
Read SHARES, not absolute lengths (stamps fence the schedule)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import mifx.ops._lib as L  # noqa: E402

# --noimg / --nostep: the builds without the weight-image load / the step-counter load (bash tools/build_stamps.sh
# --noimg / --nostep; wrong results), to split the prologue
_sfx = "_noimg" if "--noimg" in sys.argv else "_nostep" if "--nostep" in sys.argv else ""
diag = ctypes.CDLL(f"tools/bin/libwdc{_sfx}_stamps.so", mode=ctypes.RTLD_GLOBAL)
diag64 = ctypes.CDLL(f"tools/bin/libwdc64{_sfx}_stamps.so", mode=ctypes.RTLD_GLOBAL)
diag256 = ctypes.CDLL(f"tools/bin/libwdc256{_sfx}_stamps.so", mode=ctypes.RTLD_GLOBAL)
L.load.cache_clear()
_orig = L.load.__wrapped__


def _load(name):
    return {"wd_chain": diag, "wd_chain64": diag64, "wd_chain256": diag256}.get(name) or _orig(name)


L.load = _load
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402

NAMES = {1: "prologue", 2: "loop->iter", 3: "gather+fwd", 4: "loss", 5: "B0", 6: "stage5+B", 7: "dW5+dA4",
         8: "B+stage4+B", 9: "dW4+dA3", 10: "B+stage3+B", 11: "dW3+dA2", 12: "B+stage2+B", 13: "dW2+dA1",
         14: "B+stage1+B", 15: "dW1", 16: "->epi", 17: "epilogue"}
CFGS = [(4, 40, False), (8, 65536, False), (8, 65536, True)] if "--quick" in sys.argv else \
    [(4, 40, False), (8, 40, False), (4, 65536, False), (8, 128, False), (8, 65536, False), (8, 65536, True)]
for NW, batch, big in CFGS:
    t64 = NW == 4 and batch <= 64  # the T = 64 build (csrc/wd_chain64.hip)
    tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device="cuda", kernel="chain", waves=NW,
                              small_tile=t64, large_tile=big, shuffle_seed=0x5EED)
    lib = diag64 if t64 else diag256 if big else diag
    tr.set_data(synthetic_records(1 << 17, device="cuda", seed=0))
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()

    buf = (ctypes.c_ulonglong * (32 * 8))()  # g_wdc_stamps is [MAXW = 8][32]
    assert lib.mifx_wdc_stamps(buf) == 0
    st = [[buf[w * 32 + i] for i in range(32)] for w in range(NW)]
    print(f"== batch {batch} grid {tr.grid} T {tr.tile}: cycles per phase (block 0; the 2nd iteration when there is one)")
    for i in range(1, 18):
        d = [st[w][i] - st[w][i - 1] for w in range(NW)]
        print(f"  {NAMES[i]:>11}: " + " ".join(f"{x:8d}" for x in d))
    print(f"  iteration (stamp 2 -> 15), wave 0: {st[0][15] - st[0][2]}; kernel (0 -> 17): {st[0][17] - st[0][0]}")

# per-block global clock (100 MHz) of the last launch (the 8-wave B=65536 trainer above): dispatch stagger and
# block imbalance
import numpy as np  # noqa: E402

bb = (ctypes.c_ulonglong * (4096 * 3))()
assert lib.mifx_wdc_blk_stamps(bb) == 0
a = np.array(bb, dtype=np.int64).reshape(4096, 3)[:tr.grid]
t0 = a[:, 0].min()
st, pro, end = (a[:, 0] - t0) / 100.0, (a[:, 1] - a[:, 0]) / 100.0, (a[:, 2] - t0) / 100.0  # us
q = lambda v: " ".join(f"{x:7.2f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))  # noqa: E731
print(f"== per-block (grid {tr.grid}), us, percentiles 0/10/50/90/100")
print(f"  start offset: {q(st)}")
print(f"  prologue:     {q(pro)}")
print(f"  duration:     {q(end - st)}")
print(f"  end offset:   {q(end)}   kernel span {end.max():.2f} us")
order = np.argsort(st)
print("  slowest 8 blocks (id, start, dur):", [(int(i), round(float(st[i]), 2), round(float(end[i] - st[i]), 2))
                                              for i in np.argsort(-(end - st))[:8]])
print("  first 16 by start:", [int(i) for i in order[:16]])
