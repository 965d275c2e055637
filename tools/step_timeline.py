#!/usr/bin/env python3
"""Per-step GPU timeline of a rocprofv3 kernel trace (one stack in flight): steps start at the
K1 count kernel; per step the span from its first kernel's start to the next step's first start,
the summed kernel time, and the idle gaps (> --gap us) with the kernels on either side -- where
the host keeps the GPU waiting (readbacks, collectives, Python between phases).
    python tools/step_timeline.py <kernel_trace.csv> [--gap 8] [--skip 4] [--show 2]"""
import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^[\w:]*::", "", n)
    return n[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap", type=float, default=8.0, help="idle gap threshold, us")
    ap.add_argument("--skip", type=int, default=4, help="steps skipped at the start (warm-up)")
    ap.add_argument("--show", type=int, default=2, help="steps whose gaps are listed")
    ap.add_argument("--start", default="k_group_count_u8", help="kernel that starts a step")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.start in r[2]]
    steps = [rows[s:e] for s, e in zip(starts, starts[1:])]
    steps = steps[a.skip:]
    spans, busy, gaps_tot = [], [], []
    per_kernel = defaultdict(float)
    for k, st in enumerate(steps):
        t0 = st[0][0]
        nxt = starts[a.skip + k + 1]
        t1 = rows[nxt][0]
        b = 0
        end = t0
        gl = []
        for s, e, n in st:
            if s > end + a.gap * 1e3:
                gl.append((end, s))
            b += max(0, e - max(s, end))
            end = max(end, e)
            per_kernel[short(n)] += (e - s) / 1e3
        spans.append((t1 - t0) / 1e3)
        busy.append(b / 1e3)
        gaps_tot.append(sum(g[1] - g[0] for g in gl) / 1e3 + (t1 - end) / 1e3)
        if k < a.show:
            print(f"step {k}: span {spans[-1]:.1f} us, busy {busy[-1]:.1f} us")
            prev = {s: n for s, e, n in st}
            for g0, g1 in gl:
                before = max((r for r in st if r[1] <= g0), key=lambda r: r[1])
                after = min((r for r in st if r[0] >= g1), key=lambda r: r[0])
                print(f"   gap {(g1 - g0) / 1e3:7.1f} us after {short(before[2]):40s} "
                      f"before {short(after[2])}")
            print(f"   tail {(t1 - end) / 1e3:7.1f} us after {short(st[-1][2])}")
    n = len(steps)
    print(f"{n} steps: span {sum(spans) / n:.1f} us, kernels busy {sum(busy) / n:.1f} us, "
          f"idle {sum(gaps_tot) / n:.1f} us")
    for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1])[:30]:
        print(f"   {k:40s} {v / n:8.1f} us/step")


if __name__ == "__main__":
    main()
