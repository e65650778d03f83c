"""Instruction mix per loop of one kernel in a gfx950 assembly dump (hipcc --cuda-device-only -S),
using the compiler's loop annotations on the block labels: the hot tile loop of a tower kernel is
the loop with the most MFMAs. Prints, per loop, MFMA / VALU (by opcode) / AGPR moves / LDS /
VMEM / SALU counts (static: one iteration's instructions).

    python tools/loop_mix.py /tmp/k_mlp.s <mangled-kernel-name>
"""
import re
import sys
from collections import Counter, defaultdict


def main():
    asm = open(sys.argv[1]).read()
    name = sys.argv[2]
    i = asm.find("\n" + name + ":")
    j = asm.find(".Lfunc_end", i)
    body = asm[i:j].split("\n")[2:]
    cur = None
    loops = defaultdict(Counter)
    depth = {}
    for l in body:
        s = l.strip()
        m = re.match(r"^\.LBB(\w+):\s*(;.*)?$", s)
        if m:
            c = m.group(2) or ""
            h = re.search(r"Header=BB(\w+) Depth=(\d+)", c)
            if "This Loop Header" in c:
                d = re.search(r"Depth=(\d+)", c)
                cur = m.group(1)
                depth[cur] = int(d.group(1)) if d else 0
            elif h:
                cur = h.group(1)
                depth[cur] = int(h.group(2))
            elif "Parent Loop" in c:
                cur = m.group(1)
            else:
                cur = None
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        if op.startswith("v_mfma"):
            k = "mfma"
        elif op.startswith("v_accvgpr"):
            k = "acc_mov"
        elif op.startswith("v_"):
            k = "valu:" + op
        elif op.startswith("ds_"):
            k = "lds"
        elif op.startswith(("global_", "buffer_", "scratch_")):
            k = "vmem"
        elif op.startswith("s_"):
            k = "salu"
        else:
            k = op
        loops[cur][k] += 1
    best = max((x for x in loops if x), key=lambda x: loops[x]["mfma"])
    for lp in sorted((x for x in loops if x), key=lambda x: -loops[x]["mfma"])[:3]:
        c = loops[lp]
        valu = sum(v for k, v in c.items() if k.startswith("valu:"))
        print(f"loop BB{lp} depth {depth.get(lp)}: mfma {c['mfma']} valu {valu} acc_mov {c['acc_mov']} "
              f"lds {c['lds']} vmem {c['vmem']} salu {c['salu']}")
    c = loops[best]
    for k, v in c.most_common():
        if k.startswith("valu:"):
            print(f"  {v:5d} {k[5:]}")


if __name__ == "__main__":
    main()
