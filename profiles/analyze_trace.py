#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per (kernel, grid) average time and
the idle gaps between consecutive dispatches (graph-replay launch overhead).

    python profiles/analyze_trace.py gpurun_out/prof/run_kernel_trace.csv [--last N]
"""
import csv
import sys
from collections import defaultdict


def main(path, last=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if last:
        rows = rows[-last:]
    agg = defaultdict(list)
    gaps = []
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        name = r["Kernel_Name"].replace("void mx::", "").split("(")[0][:60]
        grid = (r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Grid_Size_Y", ""), r.get("Workgroup_Size_X", ""))
        agg[(name, grid)].append(e - s)
        if prev_end is not None and 0 <= s - prev_end < 50_000:
            gaps.append(s - prev_end)
        prev_end = e
    tot = sum(sum(v) for v in agg.values())
    print(f"{'kernel':60s} {'grid':>22s} {'calls':>6s} {'avg_us':>9s} {'share':>6s}")
    for (name, grid), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name:60s} {str(grid):>22s} {len(v):6d} {sum(v)/len(v)/1e3:9.2f} {100*sum(v)/tot:5.1f}%")
    if gaps:
        gaps.sort()
        print(f"gaps between dispatches: n={len(gaps)} median={gaps[len(gaps)//2]/1e3:.2f}us "
              f"mean={sum(gaps)/len(gaps)/1e3:.2f}us p90={gaps[int(len(gaps)*.9)]/1e3:.2f}us")


if __name__ == "__main__":
    last = None
    if "--last" in sys.argv:
        last = int(sys.argv[sys.argv.index("--last") + 1])
    main(sys.argv[1], last)
