"""Check that no instruction of a kernel touches a VGPR whose global_load is still in flight.

    python tools/vm_inflight_check.py <disassembly.s> <kernel symbol>...

The A-direct prefill GEMM (kernels.hip gemm_kernel AD) loads its weight fragments with inline-asm
global_load_dwordx4, which hipcc does not track: the step's explicit s_waitcnt vmcnt(N) are the only
waits for those registers, and hipcc may give the destination of an in-flight load to another value
whenever it thinks the old value dead.  This scan follows each loop body (found from its backward
branch) three times round with the in-flight loads carried over, and the straight-line code once;
vmcnt(N) retires all but the N youngest vector-memory operations (LDS-DMA copies counted).  Any
read, write or address use of an in-flight destination is reported; exit status 1 if any.
Input: llvm-objdump -d --no-show-raw-insn of the device code object (addresses in the comments).
Tooling only: no GPU, nothing under oracle/.
"""
from __future__ import annotations

import re
import sys

REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(op: str) -> set:
    out = set()
    for m in REG.finditer(op):
        if m.group(1):
            out |= set(range(int(m.group(1)), int(m.group(2)) + 1))
        else:
            out.add(int(m.group(3)))
    return out


def body(lines, name):
    head = [k for k, l in enumerate(lines) if l.rstrip().endswith("<" + name + ">:")]
    if not head:
        raise SystemExit(f"{name}: not in the disassembly")
    ins = []
    for l in lines[head[0] + 1:]:
        if l.rstrip().endswith(">:"):
            break
        if "//" not in l:
            continue
        text, comment = l.split("//", 1)
        m = re.match(r"\s*([0-9A-Fa-f]+):", comment)
        if m and text.strip():
            ins.append((int(m.group(1), 16), text.strip()))
    return ins


def scan(region, reps, pend, report):
    n_issues = 0
    for _ in range(reps):
        for _, t in region:
            mnem = t.split()[0]
            ops = t[len(mnem):]
            if mnem == "s_waitcnt" and "vmcnt" in t:
                n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
                pend[:] = pend[len(pend) - n:] if 0 < n < len(pend) else ([] if n == 0 else pend)
                continue
            live = set().union(*pend) if pend else set()
            if mnem.startswith("global_load") and "lds" not in mnem:
                dst, src = regs(ops.split(",")[0]), regs(",".join(ops.split(",")[1:]))
                if (src | dst) & live:
                    n_issues += 1
                    report(t)
                pend.append(dst)
                continue
            if "load_lds" in mnem or mnem.startswith(("buffer_load", "global_store", "buffer_store")):
                pend.append(set())
                continue
            if regs(ops) & live:
                n_issues += 1
                report(t)
    return n_issues


def main(argv):
    lines = open(argv[1]).read().split("\n")
    total = 0
    for name in argv[2:]:
        ins = body(lines, name)
        shown = []
        rep = lambda t: shown.append(t) if len(shown) < 8 else None
        issues = scan(ins, 1, [], rep)  # straight-line pass
        loops = []
        for j, (addr, t) in enumerate(ins):
            m = re.match(r"s_(?:cbranch_\w+|branch)\s+(\d+)", t)
            if m:
                off = int(m.group(1))
                off = off - 65536 if off >= 32768 else off
                if off < 0:
                    tgt = addr + 4 + 4 * off
                    h = [q for q, (a, _) in enumerate(ins) if a == tgt]
                    if h:
                        loops.append((h[0], j))
        for h, b in loops:
            issues += scan(ins[h:b + 1], 3, [], rep)
        print(f"{name}: {len(ins)} instructions, {len(loops)} loops, {issues} in-flight register uses")
        for t in shown:
            print("   ", t)
        total += issues
    return 1 if total else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
