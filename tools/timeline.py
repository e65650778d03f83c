"""One-epoch kernel timeline from a rocprofv3 --kernel-trace CSV run (the epoch between two
consecutive k_adam launches near the end of the run): start / end / duration in us and the
hardware queue, which shows the two graph branches (training chain, evaluation of the previous
epoch) and the gaps on the critical path.

Usage: python tools/timeline.py gpurun_out/prof_real2 [--back 3] > profiles/<name>.txt
"""
import argparse
import csv
from pathlib import Path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--back", type=int, default=3, help="which k_adam-to-k_adam window, from the end")
    a = ap.parse_args()
    rows = []
    for f in Path(a.dir).glob("*kernel_trace.csv"):
        rows += list(csv.DictReader(open(f)))
    for f in Path(a.dir).glob("*results.db"):          # rocpd SQLite output
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
    idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("k_adam")]
    lo, hi = idx[-a.back - 1], idx[-a.back]
    t0 = int(rows[lo]["Start_Timestamp"])
    print(f"{'start_us':>9} {'end_us':>9} {'dur_us':>8} {'queue':>5}  kernel")
    for r in rows[lo:hi + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} {r['Queue_Id']:>5}  {r['Kernel_Name'][:72]}")


if __name__ == "__main__":
    main()
