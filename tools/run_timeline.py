"""Whole timed region of a short bench run from a rocprofv3 --kernel-trace CSV: every kernel of
the last N k_adam launches' span (the timed epochs end the trace when the bench runs with
--no-ensemble9), with the gaps between consecutive kernels of the training queue, so fill /
drain costs of the per-phase graph launches (head / body / tail) show up.

Usage: python tools/run_timeline.py gpurun_out/<prof dir> [--adams 20] > profiles/<name>.txt
"""
import argparse
import csv
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--adams", type=int, default=20, help="number of trailing marker launches to cover")
    ap.add_argument("--marker", default="k_adam", help="kernel that marks an epoch (k_lstm_tail with the update in the tail)")
    a = ap.parse_args()
    rows = []
    for f in Path(a.dir).glob("**/*kernel_trace.csv"):
        rows += list(csv.DictReader(open(f)))
    for f in Path(a.dir).glob("**/*results.db"):          # rocpd SQLite output
        import sqlite3
        q = ("select s.kernel_name, d.start, d.end, d.queue_id from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        rows += [{"Kernel_Name": n, "Start_Timestamp": b, "End_Timestamp": e, "Queue_Id": str(qid)}
                 for n, b, e, qid in sqlite3.connect(str(f)).execute(q)]
    from kernel_stats import demangle
    dm = demangle({r["Kernel_Name"] for r in rows})
    for r in rows:
        r["Kernel_Name"] = dm[r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith(a.marker)]
    lo = idx[-a.adams - 1] if len(idx) > a.adams else 0
    sel = rows[lo:]
    t0 = int(sel[0]["Start_Timestamp"])
    busy_end = t0
    print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8} {'idle_us':>8} {'queue':>5}  kernel")
    idle_total = 0.0
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        idle = max(0, s - busy_end) / 1e3
        idle_total += idle
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {idle:8.1f} {r['Queue_Id']:>5}  "
              f"{r['Kernel_Name'][:70]}")
    span = (busy_end - t0) / 1e3
    print(f"# span {span:.1f} us, GPU idle (no kernel running) {idle_total:.1f} us, {len(idx[-a.adams:])} k_adam")


if __name__ == "__main__":
    main()
