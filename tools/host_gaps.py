"""Host/GPU interleaving of a short bench run: a rocprofv3 --kernel-trace --hip-trace CSV pair
merged into one timeline of the timed region (the last N k_adam launches), so every GPU idle gap
can be matched with what the host was doing (graph launches that block, event records, ...).

Usage: python tools/host_gaps.py gpurun_out/<prof dir> [--adams 21] [--min-api-us 5]
"""
import argparse
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--adams", type=int, default=21)
    ap.add_argument("--min-api-us", type=float, default=5.0)
    ap.add_argument("--marker", default="k_adam", help="kernel marking an epoch (k_lstm_tail: update in the tail)")
    a = ap.parse_args()
    kr, hr = [], []
    for f in Path(a.dir).glob("**/*kernel_trace.csv"):
        kr += list(csv.DictReader(open(f)))
    for f in Path(a.dir).glob("**/*hip_api_trace.csv"):
        hr += list(csv.DictReader(open(f)))
    from kernel_stats import demangle
    dm = demangle({r["Kernel_Name"] for r in kr})
    kr.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(kr) if dm[r["Kernel_Name"]].startswith(a.marker)]
    lo = idx[-a.adams - 1] if len(idx) > a.adams else 0
    t0, t1 = int(kr[lo]["Start_Timestamp"]), int(kr[-1]["End_Timestamp"])
    ev = []
    busy = t0
    for r in kr[lo:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        idle = max(0, s - busy) / 1e3
        busy = max(busy, e)
        ev.append((s, "K", f"{(e - s) / 1e3:7.1f} idle {idle:6.1f}  {dm[r['Kernel_Name']][:60]}"))
    tot = defaultdict(lambda: [0, 0.0])
    for r in hr:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e < t0 - 2_000_000 or s > t1:
            continue
        d = (e - s) / 1e3
        tot[r["Function"]][0] += 1
        tot[r["Function"]][1] += d
        if d >= a.min_api_us and s >= t0 - 200_000:
            ev.append((s, "H", f"{d:7.1f}          {r['Function']}"))
    ev.sort()
    for s, kind, txt in ev:
        print(f"{(s - t0) / 1e3:10.1f} {kind} {txt}")
    print("# host API totals near the timed region (calls, ms):")
    for k, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:20]:
        print(f"#   {k:40s} {n:6d} {d / 1e3:9.3f}")


if __name__ == "__main__":
    main()
