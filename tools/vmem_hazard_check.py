"""Straight-line check of hand-counted vmcnt waits in a kernel's assembly (hipcc --save-temps).

Simulates the in-order vector-memory counter over the text of one function: every VMEM load
joins the queue with its destination registers, `s_waitcnt vmcnt(N)` retires the oldest loads
until N remain, and any instruction that reads or overwrites a register of a still-pending load
is reported. Branches are ignored (the text is taken in order), which suits unrolled loop bodies.

    python tools/vmem_hazard_check.py file.s mangled_kernel_name [first_line]
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def main():
    path, name = sys.argv[1], sys.argv[2]
    first = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    pend, bad = [], 0
    for i in range(start, len(lines)):
        l = lines[i].split(";")[0].strip()
        if l.startswith(".Lfunc_end"):
            break
        if i < first or not l or l.endswith(":") or l.startswith("."):
            continue
        op, _, rest = l.partition(" ")
        toks = [t.strip() for t in re.split(r",\s*", rest) if t.strip()]
        m = re.match(r"s_waitcnt.*vmcnt\((\d+)\)", l)
        if m:
            n = int(m.group(1))
            while len(pend) > n:
                pend.pop(0)
            continue
        used = set()
        for t in toks:
            used |= regs(t.split()[0])
        for (ln, d) in pend:
            if used & d:
                print(f"line {i + 1}: {l}  touches pending load of line {ln + 1}")
                bad += 1
                break
        if op.startswith(("global_load", "buffer_load", "flat_load")) and "lds" not in op:
            pend.append((i, regs(toks[0])))
        elif op.startswith(("global_load_lds", "buffer_load")) or "lds" in op:
            pend.append((i, set()))
        elif op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic")):
            pend.append((i, set()))
    print(f"{bad} hazards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
