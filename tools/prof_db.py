#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 (ROCm 7.2 rocpd SQLite) kernel trace.

    python tools/prof_db.py <results.db> [--top 40] [--match substr] [--grid]

Groups dispatches by kernel name (and grid with --grid) and prints calls, average / min / max
duration (us), total (ms) and share, like rocprofv3's --stats CSV.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match")
    ap.add_argument("--grid", action="store_true")
    a = ap.parse_args()
    out, total = summarize(a.db, a.grid, a.match)
    print(f"{'kernel':<90} {'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'total_ms':>9} share")
    for tot, name, grid, n, avg, mn, mx in out[:a.top]:
        nm = (name[:70] + " " + grid)[-90:]
        print(f"{nm:<90} {n:>6} {avg:>9.2f} {mn:>9.2f} {mx:>9.2f} {tot / 1e3:>9.3f} {100 * tot / total:5.1f}%")


if __name__ == "__main__":
    main()
