"""Summarise a rocprofv3 kernel trace directory: per-kernel count / mean
duration, and the last N dispatches with their start gaps (host-bound
launch sequences show up as gaps larger than the kernels)."""
import csv
import glob
import os
import sys
from collections import defaultdict

d = sys.argv[1]
n_tail = int(sys.argv[2]) if len(sys.argv) > 2 else 80
f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"][:90]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{len(v):6d} {sum(v) / len(v) / 1e3:10.2f} us  {k}")
print("--- tail")
prev = None
for r in rows[-n_tail:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"gap {gap:9.2f} us  dur {(e - s) / 1e3:9.2f} us  {r['Kernel_Name'][:80]}")
    prev = e
