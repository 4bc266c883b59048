"""VALU / MFMA / LDS / accvgpr instruction counts per source line (from .loc directives) of one kernel in a
gfx950 assembly file compiled with -gline-tables-only.

    python scripts/isa_lines.py file.s kernel-substring [first-line last-line]   (assembly line range: a loop)"""
import re
import sys
from collections import Counter, defaultdict


def main(path, filt, lo=None, hi=None):
    files = {}
    cur = None
    inside = False
    loc = None
    counts = defaultdict(Counter)
    for n, line in enumerate(open(path), 1):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]+)"(?:\s+"([^"]+)")?', line)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]
        if re.match(r"^_Z\S*:", line):
            inside = filt in line
        if not inside:
            continue
        if lo is not None and not (int(lo) <= n <= int(hi)):
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            continue
        s = line.strip()
        if not s or s[0] in ";." or s.endswith(":"):
            continue
        op = s.split()[0]
        k = ("mfma" if op.startswith("v_mfma") else "acc" if op.startswith("v_accvgpr") else "valu" if op.startswith("v_")
             else "lds" if op.startswith("ds_") else "wait" if op.startswith("s_waitcnt") else None)
        if k:
            counts[loc][k] += 1
    tot = Counter()
    for c in counts.values():
        tot.update(c)
    print("total", dict(tot))
    for loc, c in sorted(counts.items(), key=lambda kv: -(kv[1]["valu"] + kv[1]["acc"]))[:40]:
        print(f"{loc:28s} valu {c['valu']:5d} acc {c['acc']:4d} mfma {c['mfma']:4d} lds {c['lds']:4d} wait {c['wait']:4d}")


if __name__ == "__main__":
    main(*sys.argv[1:])
