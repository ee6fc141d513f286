#!/usr/bin/env python3
"""Audit of hand-counted asm loads in the gemm256t kernels (guide §5.7 item 1):
between an inline-asm global load and the next inline-asm s_waitcnt, no
compiler instruction may touch the load's destination VGPRs, and the kernel
must not use scratch.  Usage: python tools/gemm_lab/audit_asm.py <gemm .s file>"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"v(\d+)", tok)
    return {int(m.group(1))} if m else set()


def audit(text: str, name: str) -> list:
    i = text.index(name + ":")
    body = text[i:text.index(".Lfunc_end", i)].splitlines()
    problems, pending, in_asm = [], {}, False
    for k, line in enumerate(body):
        s = line.strip()
        if s.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if s.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        toks = re.findall(r"v\[\d+:\d+\]|v\d+", s.split(";")[0])
        if in_asm:
            if s.startswith("global_load"):
                for r in regs(toks[0]):
                    pending[r] = k
            elif s.startswith("s_waitcnt"):
                pending.clear()
            continue
        if "scratch_" in s:
            problems.append(f"{k}: scratch access: {s}")
        used = set().union(*(regs(t) for t in toks)) if toks else set()
        hit = used & set(pending)
        if hit:
            problems.append(f"{k}: touches pending asm-load registers {sorted(hit)}: {s}")
    return problems


def main():
    text = open(sys.argv[1]).read()
    names = sorted(set(re.findall(r"^(_ZN2nr15gemm256t_kernel\w+):", text, flags=re.M)))
    bad = 0
    for n in names:
        p = audit(text, n)
        print(f"{n}: {len(p)} problem(s)")
        for x in p[:10]:
            print("   ", x)
        bad += len(p)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
