"""Print one steady-state step of a rocprofv3 kernel trace as a timeline (start/end offsets, queue).

    python scripts/prof_timeline.py <kernel_trace.csv> [--marker gather_step_kernel] [--back 20]

Useful for multi-stream graphs: shows which kernels overlap and where the GPU idles.
"""
import argparse
import csv


def load_trace(path):
    """Kernel dispatch rows {Kernel_Name, Start_Timestamp, End_Timestamp}: from rocprofv3's CSV kernel trace, or
    from its rocpd SQLite database (ROCm 7.2's default output: the ``kernels`` view)."""
    if path.endswith(".db"):
        import sqlite3
        con = sqlite3.connect(path)
        return [{"Kernel_Name": n, "Start_Timestamp": str(a), "End_Timestamp": str(b)}
                for n, a, b in con.execute("select name, start, end from kernels")]
    return list(csv.DictReader(open(path)))



def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--marker", default="gather_step_kernel")
    ap.add_argument("--back", type=int, default=20, help="which step, counted from the end")
    a = ap.parse_args()
    rows = load_trace(a.path)
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    lo, hi = idx[-a.back], idx[-a.back + 1]
    t0 = int(rows[lo]["Start_Timestamp"])
    end_max = 0
    print("| start us | end us | dur us | idle before | queue | kernel |\n|---|---|---|---|---|---|")
    for r in rows[lo:hi + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        idle = max(0, s - end_max)
        end_max = max(end_max, e)
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        print(f"| {s / 1e3:.1f} | {e / 1e3:.1f} | {(e - s) / 1e3:.1f} | {idle / 1e3:.1f} | {q} | `{r['Kernel_Name'][:70]}` |")


if __name__ == "__main__":
    main()
