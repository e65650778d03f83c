"""Static instruction mix of the HIP kernels: compile a csrc/*.hip file to gfx950 assembly and
count, per kernel and for its hottest loop (the basic-block range closed by the backward
branch with the most MFMAs), MFMA / VALU / AGPR-move / scratch / LDS / global / SALU
instructions. Used to see what a tower kernel spends its issue slots on before measuring it.

    python tools/isa_stats.py csrc/k_mlp.hip [substring-of-demangled-kernel-name ...]
"""
from __future__ import annotations

import re
import subprocess
import sys
import sysconfig
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def compile_asm(src: Path, out: Path) -> str:
    import pybind11
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{ROOT / 'csrc'}",
           f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}", "--cuda-device-only",
           "-S", str(src), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    return out.read_text()


def classify(op: str) -> str:
    if op.startswith(("scratch_", "buffer_")):
        return "scratch"
    if op.startswith("v_accvgpr"):
        return "agpr_mov"
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("global_"):
        return "global"
    return op


def functions(asm: str):
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)\n\.Lfunc_end\d+:", asm, re.S):
        yield m.group(1), m.group(2)


def stats(body: str):
    lines = [l.strip() for l in body.split("\n")]
    ins, labels = [], {}
    for l in lines:
        if not l or l.startswith((";", ".")) and not l.endswith(":"):
            continue
        if l.endswith(":") or re.match(r"^\.LBB\w+:", l):
            labels[l.split(":")[0]] = len(ins)
            continue
        ins.append(l.split(";")[0].strip())
    total = Counter(classify(i.split()[0]) for i in ins)
    best = None
    for pos, i in enumerate(ins):
        parts = i.split()
        if parts[0].startswith("s_cbranch") and len(parts) > 1 and parts[1] in labels:
            start = labels[parts[1]]
            if start <= pos:
                c = Counter(classify(x.split()[0]) for x in ins[start:pos + 1])
                if best is None or c["mfma"] > best[0]["mfma"]:
                    best = (c, start, pos)
    return total, best


def main(argv):
    src = Path(argv[1]) if len(argv) > 1 else ROOT / "csrc" / "k_mlp.hip"
    pats = argv[2:]
    asm = compile_asm(src, Path("/tmp") / (src.stem + ".s"))
    keys = ["mfma", "valu", "agpr_mov", "scratch", "lds", "global", "salu", "wait"]
    for name, body in functions(asm):
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        if pats and not any(p in dn for p in pats):
            continue
        total, best = stats(body)
        print(dn[:100])
        print("   kernel: " + " ".join(f"{k}={total[k]}" for k in keys))
        if best:
            print("   loop:   " + " ".join(f"{k}={best[0][k]}" for k in keys))


if __name__ == "__main__":
    main(sys.argv)
