"""GPU idle gaps of a rocprofv3 kernel trace (``--kernel-trace --output-format csv``): every interval where no kernel
of the traced process runs, with the kernels on both sides, and the busy / idle split of the traced window.

    python scripts/gaps.py <run_kernel_trace.csv> [min_gap_us=20] [top=25]
"""
import csv
import re
import sys


def short(name):
    m = re.search(r"(mat_\w+|\w+_kernel|\w+Kernel|\w+)(<[^>]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(path, min_gap_us=20.0, top=25):
    rows = []
    for r in csv.DictReader(open(path)):
        s, e = int(r.get("Start_Timestamp") or r["Start_Timestamp"]), int(r["End_Timestamp"])
        rows.append((s, e, short(r.get("Kernel_Name", ""))))
    rows.sort()
    if not rows:
        print("no kernels")
        return
    gaps, end, prev = [], rows[0][1], rows[0][2]
    for s, e, n in rows[1:]:
        if s > end:
            gaps.append(((s - end) / 1e3, prev, n))
        if e > end:
            end, prev = e, n
    # busy time = union of the kernel intervals
    union, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    for s, e, _ in rows[1:]:
        if s > cur_e:
            union += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    union += cur_e - cur_s
    window = rows[-1][1] - rows[0][0]
    idle = sum(g[0] for g in gaps)
    print(f"window {window / 1e6:.2f} ms, kernels busy {union / 1e6:.2f} ms, idle {idle / 1e3:.2f} ms in "
          f"{len(gaps)} gaps ({sum(1 for g in gaps if g[0] >= min_gap_us)} >= {min_gap_us} us)")
    for g, a, b in sorted(gaps, reverse=True)[:top]:
        if g < min_gap_us:
            break
        print(f"{g:9.1f} us  after {a:45s} before {b}")


if __name__ == "__main__":
    main(sys.argv[1], *(float(x) for x in sys.argv[2:3]), *(int(x) for x in sys.argv[3:4]))
