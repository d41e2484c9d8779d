"""Aggregate rocprofv3 --pmc counter_collection CSVs per kernel (mean per dispatch).

    python scripts/pmc_summary.py <dir-with-*_counter_collection.csv> [more dirs...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(path)):
                name = r.get("Kernel_Name", "?")
                cn = r.get("Counter_Name")
                if cn is None:
                    continue
                acc[name][cn].append(float(r.get("Counter_Value", 0) or 0))
    counters = sorted({c for k in acc.values() for c in k})
    print("| kernel | dispatches | " + " | ".join(counters) + " |")
    print("|---|---|" + "---|" * len(counters))
    rows = []
    for name, cs in acc.items():
        n = max(len(v) for v in cs.values())
        rows.append((name, n, [sum(cs[c]) / len(cs[c]) if cs.get(c) else float("nan") for c in counters]))
    rows.sort(key=lambda r: -r[2][0] if r[2] and r[2][0] == r[2][0] else 0)
    for name, n, vals in rows:
        print(f"| `{name[:70]}` | {n} | " + " | ".join(f"{v:.4g}" for v in vals) + " |")


if __name__ == "__main__":
    main()
