"""Per-kernel mean PMC counter values from a rocprofv3 --pmc database (counters_collection view).

usage: python tools/pmc_summary.py <results.db> [--match substr] [--out file.md]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select dispatch_id, kernel_name, grid_size, workgroup_size, counter_name, value "
                       "from counters_collection").fetchall()
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for did, kname, gs, ws, cname, val in rows:
        per[did][cname] += val
        names[did] = (re.sub(r"\(anonymous namespace\)::", "", kname)[:70], gs // max(ws, 1))
    agg = defaultdict(lambda: defaultdict(list))
    for did, cs in per.items():
        for c, v in cs.items():
            agg[names[did]][c].append(v)
    lines = []
    for (k, wg), cs in sorted(agg.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
        if a.match and a.match not in k:
            continue
        n = len(next(iter(cs.values())))
        lines.append(f"## {k} (workgroups {wg}, dispatches {n})")
        for c, v in sorted(cs.items()):
            lines.append(f"- {c}: {sum(v) / len(v):.4g}")
    out = "\n".join(lines)
    print(out)
    if a.out:
        open(a.out, "w").write(out + "\n")


if __name__ == "__main__":
    main()
