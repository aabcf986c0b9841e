#!/usr/bin/env python3
"""The traversal main loop of a kernel in the device asm (make asm -> build/rt_render.s): its text
and an instruction census by class and by basic block, with the s_waitcnt points (VERDICT r05
item 1: what a trip issues between one record's arrival and the next record's load).

The loop is the one whose header precedes the kernel's first `buffer_load_dwordx4` with an
`offset:32` operand (the third 16-B load of a record: the main loop; the wave-uniform prologue
reads through the scalar cache).  Blocks are listed in program order with their instruction
counts; a trip runs the head, then the inner-step and/or the triangle-step blocks (exec-masked:
a mixed trip runs both), then the tail.
Usage: python3 scripts/isa_loop.py ASM KERNEL_SYMBOL_PREFIX OUT_PREFIX"""
import re
import sys


def classify(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load", "s_memrealtime")):
        return "smem"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu_trans" if re.match(r"v_(rcp|rsq|sqrt|exp|log|sin|cos)_", op) else "valu"
    return "other"


def main():
    asm, sym, out = sys.argv[1], sys.argv[2], sys.argv[3]
    lines = open(asm).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.rstrip().endswith(":") or
                 (l.startswith(sym) and ": ;" in l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    ld = next(i for i, l in enumerate(body) if "buffer_load_dwordx4" in l and "offset:32" in l)
    hdr = max(i for i in range(ld) if "Loop Header" in body[i])
    label = body[hdr].split(":")[0]
    # the loop's blocks: the header and every block the assembler marks "in Loop: Header=<it>" (Depth=1)
    tag = "Header=" + label[2:]   # ".LBB51_7" -> "Header=BB51_7"
    loop, inside = [], False
    for i, l in enumerate(body):
        s_ = l.strip()
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", s_):
            inside = i == hdr or (tag in l and "Depth=1" in l)
        if inside:
            loop.append(l)
    blocks, cur = [], {"name": "(entry)", "n": 0, "cls": {}}
    waits = []
    for l in loop:
        s = l.strip()
        if re.match(r"^(\.LBB\w+|; %bb\.\d+):", s):
            blocks.append(cur)
            cur = {"name": s.split(":")[0], "n": 0, "cls": {}}
            continue
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        c = classify(op)
        cur["n"] += 1
        cur["cls"][c] = cur["cls"].get(c, 0) + 1
        if c == "waitcnt":
            waits.append(f"{cur['name']}: {s}")
    blocks.append(cur)
    tot = {}
    for b in blocks:
        for k, v in b["cls"].items():
            tot[k] = tot.get(k, 0) + v
    with open(out + ".s", "w") as f:
        f.write("\n".join(loop) + "\n")
    with open(out + ".txt", "w") as f:
        f.write(f"kernel {sym}, loop {label}: {sum(b['n'] for b in blocks)} instructions in {len(blocks)} blocks\n")
        f.write("by class: " + ", ".join(f"{k} {v}" for k, v in sorted(tot.items())) + "\n\nblocks in program order:\n")
        for b in blocks:
            f.write(f"  {b['name']:12s} {b['n']:4d}  " + ", ".join(f"{k} {v}" for k, v in sorted(b["cls"].items())) + "\n")
        f.write("\ns_waitcnt points:\n" + "\n".join("  " + w for w in waits) + "\n")
    print(open(out + ".txt").read())


if __name__ == "__main__":
    main()
