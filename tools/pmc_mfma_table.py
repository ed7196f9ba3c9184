"""MFMA utilisation per kernel from one rocprofv3 --pmc pass (counters SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE,
SQ_INSTS_MFMA, SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE): per kernel name, the dispatches, the mean
duration in cycles (GRBM_GUI_ACTIVE / 8 XCDs, counted under the profiler: short kernels read long), MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / duration, LDS instructions per MFMA and the LDS bank-conflict share; sorted by
total cycles, top N.

usage: python tools/pmc_mfma_table.py <results.db> [--top 25] [--title text] [--match regex]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--title", default="PMC: MFMA utilisation per kernel")
    ap.add_argument("--match", default=None, help="regular expression: only kernels whose name matches")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select dispatch_id, kernel_name, grid_size, workgroup_size, counter_name, value "
                       "from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for did, kname, gs, ws, cname, val in rows:
        if a.match and not re.search(a.match, kname):
            continue
        per[did][cname] += val
        names[did] = (re.sub(r"\(anonymous namespace\)::", "", kname)[:80], gs // max(ws, 1))
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for did, cs in per.items():
        k = names[did]
        cnt[k] += 1
        for c, v in cs.items():
            agg[k][c] += v
    out = [f"# {a.title}", "", "| kernel | WGs | dispatches | mean cycles | MFMA busy | LDS instr / MFMA | LDS conflict share |",
           "|---|---|---|---|---|---|---|"]
    order = sorted(agg, key=lambda k: -agg[k].get("GRBM_GUI_ACTIVE", 0.0))
    for k in order[:a.top]:
        c, n = agg[k], cnt[k]
        dur = c.get("GRBM_GUI_ACTIVE", 0.0) / 8 / n
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / 1024 / n / dur if dur else 0.0
        mf = c.get("SQ_INSTS_MFMA", 0.0)
        lds = c.get("SQ_INSTS_LDS", 0.0) / mf if mf else float("nan")
        act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / act if act else 0.0
        out.append(f"| `{k[0]}` | {k[1]} | {n} | {dur:,.0f} | {100 * busy:.0f} % | {lds:.2f} | {100 * conf:.1f} % |")
    print("\n".join(out))


if __name__ == "__main__":
    main()
