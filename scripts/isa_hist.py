"""Static instruction histogram of one kernel of a hipcc ``-S`` listing, whole kernel and its largest loop.

    hipcc ... --offload-device-only -S file.hip -o out.s
    python scripts/isa_hist.py out.s <kernel-name-substring> [top=40]

The largest loop is the span between a label and the last backward branch to it with the most instructions (for the
decode kernels: the agent loop), so the setup code does not dilute the per-iteration mix.
"""
import collections
import re
import sys

INST = re.compile(r"\s+([sv]_\w+|ds_\w+|global_\w+|buffer_\w+|flat_\w+|scratch_\w+)\b")


def kernel_lines(path, key):
    out, on = [], False
    for line in open(path):
        if re.match(r"^_Z\S+:", line):
            on = key in line.split(":")[0]
        elif on and line.startswith("\t.size"):
            break
        if on:
            out.append(line.rstrip("\n"))
    return out


def hist(lines):
    c = collections.Counter()
    for ln in lines:
        m = INST.match(ln)
        if m:
            c[m.group(1)] += 1
    return c


def largest_loop(lines):
    labels = {}
    best = (0, 0, 0)
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", ln)
        if m:
            labels[m.group(1)] = i
        m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            if any("s_endpgm" in x for x in lines[labels[m.group(2)]:i]):   # a cold block jumping back: no loop
                continue
            n = sum(1 for x in lines[labels[m.group(2)]:i + 1] if INST.match(x))
            if n > best[0]:
                best = (n, labels[m.group(2)], i + 1)
    return lines[best[1]:best[2]]


def show(title, c, top):
    tot = sum(c.values())
    cls = collections.Counter()
    for k, v in c.items():
        cls["mfma" if "mfma" in k else "valu" if k.startswith("v_") else "salu" if k.startswith("s_") else
            "lds" if k.startswith("ds_") else "vmem"] += v
    print(f"== {title}: {tot} instructions; " + ", ".join(f"{k} {v}" for k, v in cls.most_common()))
    for k, v in c.most_common(top):
        print(f"{v:7d} {k}")


if __name__ == "__main__":
    lines = kernel_lines(sys.argv[1], sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    show("kernel", hist(lines), top)
    show("largest loop", hist(largest_loop(lines)), top)
