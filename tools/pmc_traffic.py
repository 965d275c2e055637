#!/usr/bin/env python3
"""Per-launch HBM traffic of the K5 (core-flag) kernels from the rocprofv3 PMC passes of
tools/pmc.sh: bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per launch (FETCH_SIZE is in KiB and
reads half of the bytes of wide coalesced reads on gfx950, MI355X_MICROARCH.md §HBM; the factor is
calibrated for 16-B/lane streams, so for K5's narrower gathers it is an approximation).
Writes profiles/<tag>/<name> (default k5_traffic.json) and a per-kernel summary CSV."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
out_name = sys.argv[2] if len(sys.argv) > 2 else "k5_traffic.json"
workload = sys.argv[3] if len(sys.argv) > 3 else "bench.py default (100-frame stack)"
K5 = ("k_core_cells_oct", "k_core_cell_fast", "k_core_cell_window", "k_core_fill", "k_core_slow",
      "k_core_tiles")


def load(counter):
    files = glob.glob(str(ROOT / "gpurun_out" / f"pmc_{counter}" / "**" / "*counter_collection*.csv"),
                      recursive=True)
    per = defaultdict(list)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            per[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return per


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
# RPT_PROFILE_OUT: write there instead (on the GPU box: a gpurun_out/ subdirectory, the only
# place whose files come back; tools/collect_r3.sh copies them into profiles/<tag>/)
out_dir = Path(os.environ["RPT_PROFILE_OUT"]) if os.environ.get("RPT_PROFILE_OUT") else \
    ROOT / "profiles" / tag
out_dir.mkdir(parents=True, exist_ok=True)
rows = []
for name in sorted(set(fetch) | set(write)):
    f, w = fetch.get(name, []), write.get(name, [])
    fa = sum(f) / len(f) if f else 0.0
    wa = sum(w) / len(w) if w else 0.0
    rows.append((name, len(f), fa, wa, (2 * fa + wa) * 1024))
by_kernel = "pmc_traffic_by_kernel.csv" if out_name == "k5_traffic.json" else \
    out_name.replace("k5_traffic_", "pmc_traffic_by_kernel_").replace(".json", ".csv")
with open(out_dir / by_kernel, "w", newline="") as fh:
    wr = csv.writer(fh)
    wr.writerow(["kernel", "launches", "FETCH_SIZE_KiB_avg", "WRITE_SIZE_KiB_avg",
                 "hbm_bytes_per_launch_corrected"])
    for r in rows:
        wr.writerow([r[0], r[1], f"{r[2]:.1f}", f"{r[3]:.1f}", f"{r[4]:.0f}"])
k5 = {k: next((r for r in rows if k in r[0]), None) for k in K5}
total = sum(r[4] for r in k5.values() if r)
res = {"kernels": {k: (None if r is None else {"fetch_kib": r[2], "write_kib": r[3],
                                                 "bytes": r[4]}) for k, r in k5.items()},
       "bytes_per_launch": total,
       "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch, summed over the K5 kernels "
                  "that ran (" + ", ".join(k for k, r in k5.items() if r) + "); separate --pmc passes",
       "workload": workload}
(out_dir / out_name).write_text(json.dumps(res, indent=1))
print(json.dumps(res))
# K1 (the largest stage): count + group starts + expand write + the unstaged groups' write
K1 = ("k_group_count_u8", "k_group_starts", "k_expand_write", "k_group_write_u8")
k1 = [r for r in rows if any(k in r[0] for k in K1)]
if k1:
    res1 = {"kernels": {r[0][:80]: {"fetch_kib": r[2], "write_kib": r[3], "bytes": r[4]}
                        for r in k1},
            "bytes_per_launch": sum(r[4] for r in k1),
            "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch, summed over the K1 kernels",
            "workload": workload}
    (out_dir / out_name.replace("k5_", "k1_")).write_text(json.dumps(res1, indent=1))
    print(json.dumps(res1))
