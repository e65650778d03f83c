"""Per-kernel time summary from a rocprofv3 --kernel-trace run (CSV or rocpd SQLite output).

Usage: python tools/kernel_stats.py gpurun_out/prof4 [--top 30] > profiles/<name>.txt
"""
from __future__ import annotations

import argparse
import csv
import sqlite3
from collections import defaultdict
from pathlib import Path


def demangle(names):
    """Demangled kernel names (rocprofv3 writes mangled ``_Z...kd`` symbols with some options)."""
    import shutil
    import subprocess
    names = list(names)
    raw = [n[:-3] if n.endswith(".kd") else n for n in names]
    tool = shutil.which("c++filt") or "/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
    try:
        out = subprocess.run([tool], input="\n".join(raw), capture_output=True, text=True, check=True).stdout
        dem = out.split("\n")[:len(raw)]
        return dict(zip(names, dem)) if len(dem) == len(raw) else dict(zip(names, raw))
    except (OSError, subprocess.CalledProcessError):
        return dict(zip(names, raw))


def from_db(path: Path):
    c = sqlite3.connect(str(path))
    q = ("select s.kernel_name, d.end - d.start, s.arch_vgpr_count, s.accum_vgpr_count, s.sgpr_count, "
         "d.group_segment_size, d.grid_size_x, d.grid_size_y, d.grid_size_z "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    for row in c.execute(q):
        yield row[0], float(row[1]), dict(vgpr=row[2], agpr=row[3], sgpr=row[4], lds=row[5],
                                          grid=(row[6], row[7], row[8]))


def from_csv(path: Path):
    with open(path) as fh:
        for r in csv.DictReader(fh):
            yield r["Kernel_Name"], float(r["End_Timestamp"]) - float(r["Start_Timestamp"]), dict(
                vgpr=r.get("VGPR_Count"), agpr=r.get("Accum_VGPR_Count"), sgpr=r.get("SGPR_Count"),
                lds=r.get("LDS_Block_Size"), grid=r.get("Grid_Size"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    d = Path(a.dir)
    rows = []
    for f in d.glob("*results.db"):
        rows += list(from_db(f))
    for f in d.glob("*kernel_trace.csv"):
        rows += list(from_csv(f))
    agg = defaultdict(lambda: [0, 0.0, None])
    dm = demangle({r[0] for r in rows})
    for name, ns, info in rows:
        name = dm[name]
        e = agg[name]
        e[0] += 1
        e[1] += ns
        e[2] = info
    total = sum(v[1] for v in agg.values())
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}  resources")
    for name, (n, ns, info) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        short = name if len(name) <= 70 else name[:67] + "..."
        print(f"{short:70s} {n:6d} {ns / n / 1e3:9.2f} {ns / 1e6:9.3f} {100 * ns / total:6.2f}  "
              f"vgpr={info['vgpr']} agpr={info['agpr']} sgpr={info['sgpr']} lds={info['lds']}")
    print(f"total kernel time {total / 1e6:.3f} ms over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main()
