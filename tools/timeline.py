"""Dispatch timeline from a rocprofv3 --kernel-trace database: per dispatch start offset, duration and the
gap after the previous dispatch ended, for the last N dispatches matching a name filter, plus the mean
period between consecutive dispatches of the first kernel (= the step time of a replayed graph).

usage: python tools/timeline.py <results.db> [--last 12] [--match wdc_fused,wd_reduce_opt]"""
import argparse
import re
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--last", type=int, default=12)
    ap.add_argument("--match", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cols = [r[1] for r in con.execute("pragma table_info('kernels')")]
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    pats = a.match.split(",") if a.match else None
    rows = [(re.sub(r"\(anonymous namespace\)::", "", n)[:60], s, e) for n, s, e in rows
            if not pats or any(p in n for p in pats)]
    sel = rows[-a.last:]
    t0 = sel[0][1]
    prev = None
    for n, s, e in sel:
        gap = "" if prev is None else f"gap {(s - prev) / 1000:7.2f} us"
        print(f"{(s - t0) / 1000:9.2f} us  dur {(e - s) / 1000:7.2f} us  {gap}  {n}")
        prev = e
    if pats:
        first = [s for n, s, _ in rows if pats[0] in n]
        if len(first) > 10:
            per = [(b - a_) / 1000 for a_, b in zip(first[-51:-1], first[-50:])]
            print(f"period of '{pats[0]}' over the last {len(per)}: mean {sum(per) / len(per):.2f} us, "
                  f"min {min(per):.2f} us")
    print("columns:", cols[:12])


if __name__ == "__main__":
    main()
