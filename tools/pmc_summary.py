#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc counters (CSV output).

    python tools/pmc_summary.py <dir with *counter_collection.csv> [--match substr ...]

Prints, per kernel name (optionally filtered), the dispatch count and the mean value per dispatch of
every collected counter.
"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", nargs="*", default=[])
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(lambda: defaultdict(list))
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                if a.match and not any(m in name for m in a.match):
                    continue
                cn = row.get("Counter_Name") or row.get("Counter-Name")
                cv = row.get("Counter_Value") or row.get("Counter-Value")
                did = row.get("Dispatch_Id") or row.get("Dispatch-Id") or ""
                vals[name][cn].append((did, float(cv)))
    for name, cs in sorted(vals.items()):
        n = max(len({d for d, _ in v}) for v in cs.values())
        parts = []
        for cn, v in sorted(cs.items()):
            per = defaultdict(float)
            for d, x in v:
                per[d] += x
            parts.append(f"{cn}={sum(per.values()) / max(1, len(per)):.4g}")
        print(f"{name[:90]:90s} n={n} " + " ".join(parts))


if __name__ == "__main__":
    main()
