"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"| us/step | calls/step | avg us | % | kernel |\n|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    print(f"| {float(r['TotalDurationNs']) / 1e3 / steps:.1f} | {int(r['Calls']) / steps:.1f} | "
          f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / tot * 100:.1f} | `{r['Name'][:100]}` |")
print(f"\nTotal kernel time per step: {tot / 1e3 / steps:.1f} us over {sum(int(r['Calls']) for r in rows) / steps:.0f} launches")
