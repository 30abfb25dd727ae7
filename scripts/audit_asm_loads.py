#!/usr/bin/env python3
"""Audit a hipcc -save-temps .s for inline-asm register loads (global_load_dwordx4 inside
;;#ASMSTART) whose destination registers the compiler touches before the wait that retires them:
for each such load, every instruction between it and the next empty asm statement (the "+v"
hold) is scanned linearly; touches after the last s_waitcnt vmcnt before the hold are fine.

    python scripts/audit_asm_loads.py FILE.s KERNEL_SYMBOL_SUBSTRING"""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def main(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0] and ":" in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[start:end]
    bad = 0
    for i, l in enumerate(body):
        if "global_load_dwordx4" not in l or ";;#ASMSTART" not in body[i - 1]:
            continue
        dst = regs(l.split()[1].rstrip(","))
        hold = next((j for j in range(i + 1, len(body) - 1)
                     if ";;#ASMSTART" in body[j] and ";;#ASMEND" in body[j + 1]), None)
        if hold is None:
            continue
        last_wait = max((j for j in range(i, hold) if "s_waitcnt vmcnt" in body[j]), default=hold)
        for j in range(i + 1, last_wait):
            t = body[j].strip()
            if not t or t.startswith((";", ".")):
                continue
            hit = set()
            for tok in re.findall(r"v\[\d+:\d+\]|v\d+", t):
                hit |= regs(tok)
            if hit & dst and "global_load_dwordx4" not in t:
                print(f"load at {i} ({l.strip()}): touched at {j}: {t}")
                bad += 1
    print("clean" if bad == 0 else f"{bad} touches")
    return bad


if __name__ == "__main__":
    sys.exit(1 if main(sys.argv[1], sys.argv[2]) else 0)
