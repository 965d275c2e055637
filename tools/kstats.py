#!/usr/bin/env python3
"""Per-kernel average durations from a rocprofv3 --stats kernel_stats.csv (per-run calls)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 4
tot = sum(float(r["TotalDurationNs"]) for r in rows if "synth" not in r["Name"])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "synth" in r["Name"]:
        continue
    name = r["Name"].replace("void ", "").replace("rpt::(anonymous namespace)::", "")
    name = name.replace("rpt::", "").split("(")[0][:60]
    per_run = float(r["TotalDurationNs"]) / runs / 1e3
    print(f"{name:60s} calls/run={int(r['Calls']) / runs:5.1f} us/run={per_run:9.1f} "
          f"{float(r['TotalDurationNs']) / tot * 100:5.1f}%")
