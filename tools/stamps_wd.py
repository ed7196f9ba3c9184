"""Phase breakdown of wd_fused<true> block 0 via the s_memtime diagnostic build (-DWD_STAMPS).

Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -DWD_STAMPS -o tools/bin/libwd_stamps.so csrc/wide_deep.hip
Run:   python tools/stamps_wd.py      (GPU)
Read SHARES, not absolute lengths (stamps fence the schedule)."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
import mifx.ops._lib as L  # noqa: E402

diag = ctypes.CDLL("tools/bin/libwd_stamps.so", mode=ctypes.RTLD_GLOBAL)
L.load.cache_clear()
_orig = L.load.__wrapped__


def _load(name):
    return diag if name == "wide_deep" else _orig(name)


L.load = _load
from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402

NAMES = {1: "stage", 2: "fwd", 3: "loss", 4: "dA5", 5: "B1", 6: "dW5+dW4", 7: "dA4", 8: "B2", 9: "dW3",
         10: "dA3", 11: "B3", 12: "dW2", 13: "dA2", 14: "B4", 15: "dW1", 16: "B5", 17: "epilogue"}
for batch in (64, 65536):
    tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device="cuda")
    tr.set_data(synthetic_records(1 << 17, device="cuda", seed=0))
    for _ in range(3):
        tr.step()
    torch.cuda.synchronize()
    NW = 8  # waves per workgroup (csrc/wide_deep.hip NWAVE)
    buf = (ctypes.c_ulonglong * (32 * NW))()
    assert diag.mifx_wd_stamps(buf) == 0
    st = [[buf[w * 32 + i] for i in range(32)] for w in range(NW)]
    print(f"== batch {batch} grid {tr.grid}: cycles per phase (block 0, 2nd tile if any; stage = kernel start -> that tile), per wave")
    for i in range(1, 18):
        d = [st[w][i] - st[w][i - 1] for w in range(NW)]
        if i == 17:
            d = [st[w][17] - st[w][16] for w in range(NW)]
        print(f"  {NAMES[i]:>9}: " + " ".join(f"{x:8d}" for x in d))
    print(f"  total kernel (wave0 start->end): {st[0][17] - st[0][0]}")
    blk = (ctypes.c_ulonglong * 2048)()
    assert diag.mifx_wd_blk_times(blk) == 0
    nb = tr.grid
    st0 = [blk[2 * b] for b in range(nb)]
    en0 = [blk[2 * b + 1] for b in range(nb)]
    t0 = min(st0)
    starts = sorted((x - t0) / 100.0 for x in st0)  # us (100 MHz)
    ends = sorted((x - t0) / 100.0 for x in en0)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    print(f"  workgroup start us: min {starts[0]:.2f} p50 {q(starts, .5):.2f} p90 {q(starts, .9):.2f} max {starts[-1]:.2f}")
    print(f"  workgroup end   us: min {ends[0]:.2f} p50 {q(ends, .5):.2f} p90 {q(ends, .9):.2f} max {ends[-1]:.2f}")

