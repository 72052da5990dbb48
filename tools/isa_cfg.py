#!/usr/bin/env python3
"""Basic-block view of one kernel in a hipcc -S listing (ISA study aid, no GPU needed).

    python tools/isa_cfg.py listing.s KERNEL_SYMBOL [--dump BB...]

Prints every basic block with its instruction counts by class (VALU, SALU, VMEM, LDS,
scratch, readlane/writelane, waitcnt/nop, branch) and its successors, so the instruction
path of one main-loop iteration can be read off (node step, leaf step, return).
"""
import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith("s_endpgm"))
    out, cur, name = [], [], "ENTRY"
    for l in lines[start + 1:end + 1]:
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            out.append((name, cur))
            name, cur = m.group(1), []
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        cur.append(t)
    out.append((name, cur))
    return out


def klass(ins):
    op = ins.split()[0]
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sym = sys.argv[1], sys.argv[2]
    dump = set(sys.argv[sys.argv.index("--dump") + 1:]) if "--dump" in sys.argv else set()
    bbs = blocks(path, sym)
    names = [b[0] for b in bbs]
    for k, (name, ins) in enumerate(bbs):
        c = {}
        for i in ins:
            c[klass(i)] = c.get(klass(i), 0) + 1
        succ = []
        for i in ins:
            m = re.match(r"s_c?branch\w*\s+(\.LBB\w+)", i)
            if m:
                succ.append(m.group(1))
        if not (ins and ins[-1].startswith("s_branch")) and k + 1 < len(names):
            succ.append(names[k + 1] + "(ft)")
        print(f"{name:14s} n={len(ins):4d} " + " ".join(f"{kk}={v}" for kk, v in sorted(c.items())) + "  -> " + ",".join(succ))
        if name in dump:
            for i in ins:
                print("      " + i)


if __name__ == "__main__":
    main()
