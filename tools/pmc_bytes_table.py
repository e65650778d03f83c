"""Per-kernel HBM bytes from two rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE, KiB per
dispatch): mean KiB per call, calls, mean duration and the implied bandwidth.

    python tools/pmc_bytes_table.py <fetch pass dir> <write pass dir>
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(d, counter):
    per = defaultdict(list)
    for f in Path(d).rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            per[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    dur = defaultdict(list)
    for f in Path(d).rglob("*kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def main():
    fe, dur = load(sys.argv[1], "FETCH_SIZE")
    wr, _ = load(sys.argv[2], "WRITE_SIZE")
    rows = []
    for k in set(fe) | set(wr):
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        d = dur.get(k, [])
        us = sum(d) / len(d) if d else float("nan")
        rows.append((f + w, k, f, w, len(fe.get(k, [])), us))
    rows.sort(reverse=True)
    print(f"{'kernel':70s} {'calls':>5s} {'fetch MiB':>10s} {'write MiB':>10s} {'avg us':>9s} {'GB/s':>8s}")
    for tot, k, f, w, n, us in rows[:40]:
        bw = (f + w) * 1024 / (us * 1e-6) / 1e9 if us == us and us > 0 else float("nan")
        print(f"{k[:70]:70s} {n:5d} {f / 1024:10.1f} {w / 1024:10.1f} {us:9.1f} {bw:8.0f}")


if __name__ == "__main__":
    main()
