"""VGPR / scratch / LDS of every kernel in the device assembly of each translation unit (make asm TU=...).
usage: python tools/kernel_regs.py <pkg dir> [<other pkg dir>]  -> one line per kernel (and the other's figures)"""
import os
import re
import subprocess
import sys


def regs(pkg):
    out = {}
    for f in sorted(os.listdir(os.path.join(pkg, "csrc"))):
        if not f.endswith(".hip"):
            continue
        tu = f[:-4]
        subprocess.run(["make", "-s", "-C", pkg, "asm", f"TU={tu}"], check=True, capture_output=True)
        s = open(os.path.join(pkg, "build", tu + ".s")).read()
        for b in s.split("- .agpr_count")[1:]:
            n = re.search(r"\.name:\s+(\S+)", b).group(1)
            g = lambda k: int(re.search(rf"\.{k}:\s+(\d+)", b).group(1))  # noqa: E731
            out[n] = (g("vgpr_count"), g("private_segment_fixed_size"), g("group_segment_fixed_size"))
    return out


a = regs(sys.argv[1])
b = regs(sys.argv[2]) if len(sys.argv) > 2 else {}
for n in sorted(a):
    o = b.get(n)
    flag = "" if o is None or o[:2] == a[n][:2] else "   <-- " + str(o)
    print(f"{a[n][0]:4d} {a[n][1]:5d} {a[n][2]:6d}  {n[:90]}{flag}")
