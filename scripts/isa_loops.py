"""Loops (backward branches) of one kernel in a gfx950 assembly file with their static instruction mix.

    python scripts/isa_loops.py dec_bwd.s kernel-name-filter"""
import re
import sys
from collections import Counter

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_mix import classify, kernels  # noqa: E402


def main(path, filt):
    for name, body in kernels(path):
        if filt not in name:
            continue
        labels = {}
        insts = []   # (line index, op, text)
        for i, line in enumerate(body):
            s = line.strip()
            m = re.match(r"^(\.LBB\w+):", s)
            if m:
                labels[m.group(1)] = len(insts)
                continue
            if not s or s[0] in ";.":
                continue
            insts.append((i, s.split()[0], s))
        loops = []
        for k, (_, op, s) in enumerate(insts):
            if op.startswith("s_cbranch") or op == "s_branch":
                tgt = s.split()[-1]
                if tgt in labels and labels[tgt] <= k:
                    loops.append((labels[tgt], k, tgt))
        print(name[:100], "instructions:", len(insts))
        for a, b, tgt in loops:
            c = Counter(classify(op) for _, op, _ in insts[a:b + 1])
            v = Counter(op for _, op, _ in insts[a:b + 1] if classify(op) == "valu")
            print(f"  loop {tgt} [{a}, {b}] n={b - a + 1}: " + " ".join(f"{k}={c[k]}" for k in ("mfma", "valu", "lds", "vmem", "scratch", "waitcnt", "barrier", "salu")))
            print("     " + ", ".join(f"{o}:{n}" for o, n in v.most_common(10)))


if __name__ == "__main__":
    main(*sys.argv[1:])
