#!/usr/bin/env python3
"""Per-kernel mean of several tools/kstats.py summaries (same format out, for kab_diff.py).
   python tools/kab_mean.py a.txt b.txt ..."""
import re
import sys

acc, calls = {}, {}
for f in sys.argv[1:]:
    for line in open(f):
        m = re.match(r'(.+?)\s+calls/run=\s*([\d.]+)\s+us/run=\s*([\d.]+)', line)
        if m:
            k = m.group(1).strip()
            acc[k] = acc.get(k, 0.0) + float(m.group(3)) / (len(sys.argv) - 1)
            calls[k] = float(m.group(2))
tot = sum(acc.values()) or 1.0
for k in sorted(acc, key=lambda k: -acc[k]):
    print(f"{k:60s} calls/run={calls[k]:5.1f} us/run={acc[k]:9.1f} {acc[k] / tot * 100:5.1f}%")
