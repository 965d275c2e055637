#!/usr/bin/env python3
"""Per-kernel difference of two tools/kstats.py summaries (new vs base): totals and the kernels
that moved most.   python tools/kab_diff.py new.txt base.txt [top]"""
import re
import sys


def load(f):
    d = {}
    for line in open(f):
        m = re.match(r'(.+?)\s+calls/run=\s*([\d.]+)\s+us/run=\s*([\d.]+)', line)
        if m:
            d[m.group(1).strip()] = float(m.group(3))
    return d


a, b = load(sys.argv[1]), load(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 10
print(f"total {sum(a.values()):.1f} vs {sum(b.values()):.1f} us")
for k in sorted(set(a) | set(b), key=lambda k: -abs(a.get(k, 0) - b.get(k, 0)))[:top]:
    print(f"  {k[:44]:44s} {a.get(k, 0):9.1f} {a.get(k, 0) - b.get(k, 0):+8.1f}")
