#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 (ROCm 7.2 rocpd SQLite) kernel trace.

    python tools/prof_db.py <results.db> [--top 40] [--match substr] [--grid] [--gaps]

Groups dispatches by kernel name (and grid with --grid) and prints calls, average / min / max
duration (us), total (ms) and share, like rocprofv3's --stats CSV.  --gaps: the idle time between
consecutive dispatches (start of one minus end of the one before, in trace order), per (previous ->
next) kernel pair -- what a kernel boundary costs on top of the kernels' own durations.
"""
import argparse
import sqlite3
from collections import defaultdict


def summarize(path, by_grid=False, match=None):
    db = sqlite3.connect(path)
    rows = db.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels").fetchall()
    g = defaultdict(list)
    for name, dur, gx, gy, gz, wx in rows:
        if match and match not in name:
            continue
        key = (name, f"[{gx}x{gy}x{gz}]/{wx}" if by_grid else "")
        g[key].append(dur / 1000.0)
    total = sum(sum(v) for v in g.values()) or 1.0
    out = []
    for (name, grid), v in g.items():
        out.append((sum(v), name, grid, len(v), sum(v) / len(v), min(v), max(v)))
    out.sort(reverse=True)
    return out, total


def _short(name):
    n = name.split("(")[0].replace("void ", "").replace("mx::", "")
    return n[:48]


def gaps(path, match=None, top=30):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    g = defaultdict(list)
    for (pn, ps, pe), (n, s, e) in zip(rows, rows[1:]):
        if match and match not in n:
            continue
        gap = (s - pe) / 1000.0
        if 0 <= gap < 50:  # larger gaps are host-side pauses (syncs), not boundaries
            g[(_short(pn), _short(n))].append(gap)
    out = sorted(((sum(v), k, len(v), sum(v) / len(v), min(v)) for k, v in g.items()), reverse=True)
    print(f"{'previous -> next':<100} {'n':>6} {'avg_us':>8} {'min_us':>8} {'total_ms':>9}")
    for tot, (a, b), n, avg, mn in out[:top]:
        print(f"{(a + ' -> ' + b)[:100]:<100} {n:>6} {avg:>8.2f} {mn:>8.2f} {tot / 1e3:>9.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match")
    ap.add_argument("--grid", action="store_true")
    ap.add_argument("--gaps", action="store_true")
    a = ap.parse_args()
    if a.gaps:
        return gaps(a.db, a.match, a.top)
    out, total = summarize(a.db, a.grid, a.match)
    print(f"{'kernel':<90} {'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'total_ms':>9} share")
    for tot, name, grid, n, avg, mn, mx in out[:a.top]:
        nm = (name[:70] + " " + grid)[-90:]
        print(f"{nm:<90} {n:>6} {avg:>9.2f} {mn:>9.2f} {mx:>9.2f} {tot / 1e3:>9.3f} {100 * tot / total:5.1f}%")


if __name__ == "__main__":
    main()
