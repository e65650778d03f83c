"""Summarise rocprofv3 counter-collection CSVs per kernel.

Usage: python tools/pmc_summary.py gpurun_out/pmc1 gpurun_out/pmc2 > profiles/<name>.txt

Prints, per kernel (top by dispatch count x grid), the mean of every collected counter per
dispatch and per wave (SQ_WAVES normalised), plus the VGPR/AGPR/SGPR/LDS resources.
"""
from __future__ import annotations

import csv
import sys
from collections import defaultdict
from pathlib import Path


def load(dirs):
    per = defaultdict(lambda: defaultdict(list))
    res = {}
    for d in dirs:
        for f in Path(d).glob("*counter_collection.csv"):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    k = r["Kernel_Name"]
                    if k.startswith("__amd") or k.startswith("void at::") or k.startswith("at::"):
                        continue
                    per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    res[k] = (r["Grid_Size"], r["Workgroup_Size"], r["VGPR_Count"], r["Accum_VGPR_Count"],
                              r["SGPR_Count"], r["LDS_Block_Size"], r["Scratch_Size"])
    return per, res


def main(argv):
    per, res = load(argv[1:] or ["gpurun_out/pmc1"])
    for k in sorted(per):
        c = per[k]
        g, wg, v, a, s, lds, scr = res[k]
        print(f"== {k}\n   grid={g} wg={wg} vgpr={v} agpr={a} sgpr={s} lds={lds} scratch={scr}")
        waves = None
        if "SQ_WAVES" in c:
            waves = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"])
        for name in sorted(c):
            vals = c[name]
            m = sum(vals) / len(vals)
            pw = f"  per-wave={m / waves:12.1f}" if waves and name != "SQ_WAVES" else ""
            print(f"   {name:28s} mean/disp={m:16.1f}{pw}  (n={len(vals)})")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
