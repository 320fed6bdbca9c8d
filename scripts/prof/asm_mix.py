#!/usr/bin/env python3
"""Instruction mix of the MFMA loop(s) of each kernel in a hipcc -S listing (gfx950).

  hipcc --offload-arch=gfx950 -O3 -S --cuda-device-only k.hip -o k.s && python scripts/prof/asm_mix.py k.s [regex]

For every kernel matching the regex: the innermost backward-branch loop that contains MFMAs,
with its VALU / MFMA / vector-memory / LDS / v_mov counts (a quick VALU:MFMA ratio check before
spending GPU time)."""
import re
import sys
from collections import Counter


def loops(lines):
    """(start, end) line ranges closed by a backward branch (rotated loops: the branch target
    may sit above a body that starts at an earlier label jumped to from below)."""
    lab = {l[:-1]: i for i, l in enumerate(lines) if l.endswith(":")}
    for i, l in enumerate(lines):
        if l.startswith(("s_cbranch", "s_branch")):
            tgt = l.split()[-1]
            if tgt in lab and lab[tgt] < i:
                yield lab[tgt], i


def main():
    s = open(sys.argv[1]).read()
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    for name in re.findall(r"^(_Z\S+):", s, re.M):
        if pat and not pat.search(name):
            continue
        body = s[s.index(name + ":"):]
        end = body.find(".Lfunc_end")
        body = body[:end if end > 0 else None]
        L = [l.split(";")[0].strip() for l in body.splitlines()]
        L = [l for l in L if l and not l.startswith("//")]
        L = [l for l in L if l.endswith(":") or not l.startswith(".")]
        best = None
        for a, b in loops(L):
            if any("mfma" in x for x in L[a:b]) and (best is None or b - a < best[1] - best[0]):
                best = (a, b)
        if best is None:
            continue
        c = Counter(x.split()[0] for x in L[best[0] + 1:best[1] + 1] if not x.endswith(":"))
        mf = sum(v for k, v in c.items() if "mfma" in k)
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        vmem = sum(v for k, v in c.items() if k.startswith(("buffer_", "global_")))
        lds = sum(v for k, v in c.items() if k.startswith("ds_"))
        mov = sum(v for k, v in c.items() if k.startswith(("v_mov", "v_accvgpr")))
        print(f"{name[:90]}\n  loop {best[1] - best[0]} lines: mfma {mf}  valu {valu} (mov {mov})  vmem {vmem}  lds {lds}"
              f"  valu/mfma {valu / max(1, mf):.1f}")
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(14)))


if __name__ == "__main__":
    main()
