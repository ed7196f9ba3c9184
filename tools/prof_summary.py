"""Summarise a rocprofv3 kernel-trace database: per (kernel, grid) count / mean / total µs.

usage: python tools/prof_summary.py <results.db> [--match substr ...] [--out profiles/x.md]
"""
import argparse
import re
import sqlite3
from collections import defaultdict


def short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    m = re.match(r"(?:void )?([\w:<>, ]+?)(\(|$)", name)
    s = m.group(1) if m else name
    return s[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", nargs="*", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--title", default="rocprofv3 kernel summary")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, grid_x, workgroup_x, duration, vgpr_count, accum_vgpr_count, lds_size "
                       "from kernels").fetchall()
    agg = defaultdict(list)
    meta = {}
    for name, gx, wx, dur, vg, ag, lds in rows:
        s = short(name)
        if a.match and not any(m in s for m in a.match):
            continue
        key = (s, gx // max(wx, 1))
        agg[key].append(dur / 1000.0)
        meta[key] = (vg, ag, lds)
    tot = sum(sum(v) for v in agg.values())
    lines = [f"# {a.title}", "", "| kernel | workgroups | calls | mean µs | min µs | total µs | % | vgpr/agpr | LDS B |",
             "|---|---|---|---|---|---|---|---|---|"]
    for key, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        vg, ag, lds = meta[key]
        lines.append(f"| `{key[0]}` | {key[1]} | {len(v)} | {sum(v) / len(v):.2f} | {min(v):.2f} | {sum(v):.1f} | "
                     f"{100 * sum(v) / tot:.1f} | {vg}/{ag} | {lds} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
