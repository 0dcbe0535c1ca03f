#!/usr/bin/env python3
"""Summarise rocprofv3 output (rocpd SQLite .db or CSV directory) into committed text.

    tools/prof_summary.py stats <db-or-dir>            per-kernel calls / avg / total (kernel-trace --stats)
    tools/prof_summary.py pmc <db-or-dir> [...]        per-kernel mean of each counter per dispatch
    tools/prof_summary.py traffic <fetch> <write> <kernel> <out.json> <label>   bench.py roofline.traffic

FETCH_SIZE is reported raw (KiB, as rocprofv3 computes it) and as HBM bytes after the
gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so bytes = 2 * 1024 * KiB.
WRITE_SIZE is exact for 16-B-per-lane stores: bytes = 1024 * KiB.
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sqlite3
import sys


def _db(path):
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        if dbs:
            return sqlite3.connect(dbs[0])
        return None
    return sqlite3.connect(path)


def stats(path, by_grid=False):
    con = _db(path)
    agg = collections.defaultdict(list)
    if con is not None:
        for name, s, e, gx, gy in con.execute("select name, start, end, grid_x, grid_y from kernels"):
            agg[f"{name} [{gx}x{gy}]" if by_grid else name].append(e - s)
    else:
        for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    tot = sum(sum(v) for v in agg.values())
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    print(f"{'kernel':100s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'total_ms':>9s} {'share':>6s}")
    for name, d in rows:
        print(f"{name[-100:]:100s} {len(d):6d} {sum(d)/len(d)/1e3:9.2f} {min(d)/1e3:9.2f} {max(d)/1e3:9.2f} "
              f"{sum(d)/1e6:9.3f} {100*sum(d)/tot:5.1f}%")


def pmc(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        con = _db(path)
        for name, cn, v in con.execute("select kernel_name, counter_name, value from counters_collection"):
            agg[name][cn].append(v)
    print(f"{'kernel':100s} {'counter':12s} {'n':>5s} {'mean_KiB':>12s} {'HBM_MB/launch':>14s}")
    for name in sorted(agg, key=lambda n: -max(sum(v) for v in agg[n].values())):
        for cn, v in sorted(agg[name].items()):
            m = sum(v) / len(v)
            byt = m * 1024 * (2 if cn == "FETCH_SIZE" else 1)
            print(f"{name[-100:]:100s} {cn:12s} {len(v):5d} {m:12.1f} {byt/1e6:14.3f}")


def traffic(fetch_dir, write_dir, kernel, out, label):
    """HBM bytes per launch of one kernel (FETCH corrected x2, WRITE exact) -> JSON for bench.py."""
    import json

    vals = {}
    for path, cn in ((fetch_dir, "FETCH_SIZE"), (write_dir, "WRITE_SIZE")):
        con = _db(path)
        v = [r[0] for r in con.execute("select value from counters_collection where kernel_name = ? and counter_name = ?",
                                       (kernel, cn))]
        if not v:
            raise SystemExit(f"no {cn} samples for {kernel}")
        vals[cn] = (sum(v) / len(v), len(v))
    rec = {"kernel": kernel, "label": label,
           "fetch_bytes": vals["FETCH_SIZE"][0] * 1024 * 2, "write_bytes": vals["WRITE_SIZE"][0] * 1024,
           "dispatches": vals["FETCH_SIZE"][1],
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over bench.py; FETCH_SIZE x2 "
                     "(gfx950 correction, MI355X_MICROARCH.md HBM section), KiB x 1024"}
    rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[label] = rec
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], by_grid=len(sys.argv) > 3 and sys.argv[3] == "grid")
    elif sys.argv[1] == "traffic":
        traffic(*sys.argv[2:7])
    else:
        pmc(sys.argv[2:])
