#!/usr/bin/env python3
"""Summary of a tools/pmc_sq.sh pass: per kernel (mean over launches) waves, VALU and LDS
instructions per wave, and the VALU-active share of the wave cycles."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
rows = []
for k, c in acc.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    rows.append((m.get("SQ_WAVE_CYCLES", 0.0), k, m))
rows.sort(reverse=True)
print(f"{'kernel':44s} {'waves':>9s} {'wavecyc':>11s} {'busycyc':>10s} {'valu/w':>8s} "
      f"{'lds/w':>7s} {'vmem/w':>7s} {'salu/w':>7s} {'valu_act/wavecyc':>16s}")
for wc, k, m in rows[:25]:
    w = max(m.get("SQ_WAVES", 1.0), 1.0)
    print(f"{k[:44]:44s} {m.get('SQ_WAVES', 0):9.0f} {wc:11.3e} {m.get('SQ_BUSY_CYCLES', 0):10.3e} "
          f"{m.get('SQ_INSTS_VALU', 0) / w:8.1f} {m.get('SQ_INSTS_LDS', 0) / w:7.1f} "
          f"{m.get('SQ_INSTS_VMEM_RD', 0) / w:7.1f} {m.get('SQ_INSTS_SALU', 0) / w:7.1f} "
          f"{m.get('SQ_ACTIVE_INST_VALU', 0) / max(wc, 1.0):16.3f}")
