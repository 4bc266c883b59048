"""Static instruction mix of every kernel in a gfx950 assembly file (hipcc --cuda-device-only -S).

    python scripts/isa_mix.py dec_bwd.s [name-filter]

Per kernel: VGPR / SGPR spills and scratch, and counts of MFMA, VALU (v_* other than MFMA / accvgpr moves), accvgpr
moves, LDS (ds_*), global / buffer / scratch memory, s_waitcnt and s_barrier instructions."""
import re
import sys
from collections import Counter


def kernels(path):
    cur, body = None, []
    for line in open(path):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if cur:
                yield cur, body
            cur, body = m.group(1), []
            continue
        if cur and line.startswith("\t.size\t" + cur):
            yield cur, body
            cur, body = None, []
            continue
        if cur:
            body.append(line)


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_") or op.startswith("buffer_store") and "off" in op:
        return "scratch"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return None


def main(path, filt=""):
    for name, body in kernels(path):
        if filt not in name:
            continue
        c = Counter()
        ops = Counter()
        for line in body:
            s = line.strip()
            if not s or s[0] in ";." or s.endswith(":"):
                continue
            op = s.split()[0]
            k = classify(op)
            if k:
                c[k] += 1
                if k == "valu":
                    ops[op] += 1
        print(name[:110])
        print("  " + "  ".join(f"{k}={c[k]}" for k in ("mfma", "valu", "accmov", "lds", "vmem", "scratch", "waitcnt", "barrier", "salu")))
        print("  top VALU: " + ", ".join(f"{o}:{n}" for o, n in ops.most_common(24)))


if __name__ == "__main__":
    main(*sys.argv[1:])
