#!/usr/bin/env python3
"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals over the span from
the first to the last kernel whose name matches (default: every rpt kernel except the synthetic
echo generator), plus the largest idle gaps.  Usage: python tools/busy.py kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
iv = []
for r in rows:
    name = r.get("Kernel_Name") or r.get("Name") or ""
    if "synth" in name:
        continue
    iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
iv.sort()
# skip the warm-up: start at the 2nd k_group_count launch
starts = [i for i, v in enumerate(iv) if "k_group_count" in v[2]]
if len(starts) > 1:
    iv = iv[starts[1]:]
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s, e, n in iv[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, n))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms ({busy / (t1 - t0) * 100:.1f} %), "
      f"{len(gaps)} gaps, idle {sum(g for g, _ in gaps) / 1e6:.3f} ms")
for g, n in sorted(gaps, reverse=True)[:12]:
    print(f"  gap {g / 1e3:8.1f} us before {n[:70]}")
