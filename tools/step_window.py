"""Per-step kernel census from a rocprofv3 --kernel-trace database: the dispatches between two consecutive occurrences
of a step-marker kernel (default: the optimizer, sgd_chunks), counted and summed per kernel name, plus the summed idle
gaps -- to compare two configurations of the same step (e.g. the single-GPU and the forced one-rank DP ResNet step).

usage: python tools/step_window.py <results.db> [--marker sgd_chunks] [--which -2]"""
import argparse
import re
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="sgd_chunks")
    ap.add_argument("--which", type=int, default=-2, help="window index among marker occurrences (python indexing)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than 2 '{a.marker}' dispatches")
    w = list(range(len(marks) - 1))[a.which]
    i0, i1 = marks[w] + 1, marks[w + 1] + 1  # (after one optimizer) .. (through the next)
    sel = rows[i0:i1]
    agg = defaultdict(lambda: [0, 0.0])
    gaps, busy, prev = 0.0, 0.0, None
    for n, s, e in sel:
        k = re.sub(r"\(anonymous namespace\)::", "", n)[:80]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1000
        busy += (e - s) / 1000
        if prev is not None and s > prev:
            gaps += (s - prev) / 1000
        prev = max(prev or e, e)
    span = (sel[-1][2] - sel[0][1]) / 1000
    print(f"step window {w}: {len(sel)} dispatches, span {span:.1f} us, kernel time {busy:.1f} us, idle gaps {gaps:.1f} us")
    print("| kernel | calls | total us |")
    print("|---|---|---|")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"| `{k}` | {c} | {t:.1f} |")


if __name__ == "__main__":
    main()
