#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of librtamd's device code.

Compiles csrc/rt_render.hip for gfx950 with -Rpass-analysis=kernel-resource-usage (the
Makefile's `asm` target) and prints one line per kernel: demangled-ish name, VGPRs, AGPRs,
SGPRs, scratch bytes per lane, LDS bytes, waves per SIMD.  Usage:
    python3 scripts/resource_usage.py [filter-substring] [-- extra make args, e.g. KDEFS=-DX=1]
"""
import os
import re
import subprocess
import sys

PKG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "real-time-opencl-raytracer_amd")


def main():
    args = sys.argv[1:]
    extra = []
    if "--" in args:
        i = args.index("--")
        args, extra = args[:i], args[i + 1:]
    filt = args[0] if args else ""
    out = subprocess.run(["make", "-s", "asm", *extra], cwd=PKG, capture_output=True, text=True)
    cur, rows = None, []
    for line in (out.stdout + out.stderr).splitlines():
        m = re.search(r"remark: (.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        key, val = m.group(1).strip(), m.group(2).strip()
        if key == "Function Name":
            cur = {"name": val}
            rows.append(cur)
        elif cur is not None:
            cur[key] = val
    for r in rows:
        n = r["name"]
        if filt and filt not in n:
            continue
        short = re.sub(r"EEEvN3rtk.*$", "", n)
        short = short.replace("_ZN", "").replace("ILb", "<").replace("ELb", ",").replace("ELi", ",i")
        print(f"{short:60s} vgpr {r.get('VGPRs', '?'):>3} agpr {r.get('AGPRs', '?'):>3} sgpr {r.get('SGPRs', '?'):>3} "
              f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>3} lds {r.get('LDS Size [bytes/block]', '?'):>6} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main()
