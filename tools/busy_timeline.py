"""GPU busy fraction over time from a rocprofv3 kernel trace (--kernel-trace, csv): the union of
all kernels' [start, end) intervals, per 1 ms bin, and the idle gaps longer than 50 us.

    python tools/busy_timeline.py <kernel_trace.csv> [t_from_ms] [t_to_ms]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in rows)
    t0 = iv[0][0]
    lo = float(sys.argv[2]) * 1e6 + t0 if len(sys.argv) > 2 else t0
    hi = float(sys.argv[3]) * 1e6 + t0 if len(sys.argv) > 3 else iv[-1][1]
    merged = []
    for s, e, _ in iv:
        if e < lo or s > hi:
            continue
        s, e = max(s, lo), min(e, hi)
        if merged and s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    busy = sum(e - s for s, e in merged)
    span = hi - lo
    print(f"window {span / 1e6:.2f} ms, busy {busy / 1e6:.2f} ms ({100 * busy / span:.1f} %)")
    gaps = [(merged[k][1], merged[k + 1][0]) for k in range(len(merged) - 1)
            if merged[k + 1][0] - merged[k][1] > 50_000]
    tot = sum(b - a for a, b in gaps)
    print(f"{len(gaps)} idle gaps > 50 us, {tot / 1e6:.2f} ms in total")
    for a, b in gaps[:40]:
        print(f"  idle {(a - t0) / 1e6:9.3f} .. {(b - t0) / 1e6:9.3f} ms ({(b - a) / 1e3:7.1f} us)")


if __name__ == "__main__":
    main()
