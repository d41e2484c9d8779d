"""Summarise rocprofv3 output: top kernels per training step.

    python scripts/prof_summary.py <kernel_stats.csv> [steps] [top]
    python scripts/prof_summary.py <kernel_trace.csv> [--marker 'conv3x3_kernel<2,'] [--per-step 2] [--tail 0.5] [--top 40]

With a kernel *trace*, only the steady-state tail of the run is used (the last ``--tail``
fraction of dispatches by start time, so data generation / warm-up / graph capture drop out)
and the step count is the number of ``--marker`` kernel dispatches in that window divided by
``--per-step`` (how many times the marker kernel runs per step).  Also reports GPU busy time
per step and the wall-clock span per step inside the window.
"""
import argparse
import csv
from collections import defaultdict


def load_trace(path):
    """Kernel dispatch rows {Kernel_Name, Start_Timestamp, End_Timestamp}: from rocprofv3's CSV kernel trace, or
    from its rocpd SQLite database (ROCm 7.2's default output: the ``kernels`` view)."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": str(a), "End_Timestamp": str(b)}
                for n, a, b in con.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))



def from_stats(path, steps, top):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print("| us/step | calls/step | avg us | % | kernel |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        print(f"| {float(r['TotalDurationNs']) / 1e3 / steps:.1f} | {int(r['Calls']) / steps:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / tot * 100:.1f} | `{r['Name'][:100]}` |")
    print(f"\nTotal kernel time per step: {tot / 1e3 / steps:.1f} us over "
          f"{sum(int(r['Calls']) for r in rows) / steps:.0f} launches")


def from_trace(path, marker, per_step, tail, top):
    rows = load_trace(path)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[int(len(rows) * (1 - tail)):]
    # start the window at a marker so partial steps at the edge do not skew the counts
    first = next(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
    last = max(i for i, r in enumerate(rows) if marker in r["Kernel_Name"])
    rows = rows[first:last + 1]
    n_mark = sum(marker in r["Kernel_Name"] for r in rows)
    steps = max((n_mark - 1) / per_step, 1)
    agg = defaultdict(lambda: [0, 0.0])
    for r in rows:
        a = agg[r["Kernel_Name"]]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    span = int(rows[-1]["Start_Timestamp"]) - int(rows[0]["Start_Timestamp"])
    # union of the kernel intervals: with a multi-stream graph kernels overlap, so the sum of
    # kernel times ("kernel time") exceeds the time the GPU had any kernel running ("busy")
    busy, cur_s, cur_e = 0, None, None
    for r in rows:
        s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_e is None or s0 > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s0, e0
        else:
            cur_e = max(cur_e, e0)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f"steady-state window: {steps:.0f} steps, wall {span / 1e3 / steps:.1f} us/step, "
          f"GPU busy (interval union) {busy / 1e3 / steps:.1f} us/step, summed kernel time "
          f"{tot / 1e3 / steps:.1f} us/step (overlap x{tot / max(busy, 1):.2f}), "
          f"{sum(v[0] for v in agg.values()) / steps:.0f} launches/step\n")
    print("| us/step | calls/step | avg us | % | kernel |\n|---|---|---|---|---|")
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"| {t / 1e3 / steps:.1f} | {c / steps:.2f} | {t / c / 1e3:.1f} | {t / tot * 100:.1f} | `{name[:110]}` |")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("steps", nargs="?", type=float, default=1.0)
    ap.add_argument("top_pos", nargs="?", type=int, default=None)
    # (the layer-1 conv forward runs once per step in every plan; the batch gather runs twice per step in the indep plan)
    ap.add_argument("--marker", default="conv3x3_kernel<2,")
    ap.add_argument("--per-step", type=float, default=1.0)
    ap.add_argument("--tail", type=float, default=0.5)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    top = a.top_pos or a.top
    if "trace" in a.path or a.path.endswith(".db"):
        from_trace(a.path, a.marker, a.per_step, a.tail, top)
    else:
        from_stats(a.path, a.steps, top)


if __name__ == "__main__":
    main()
