"""Per-kernel table from rocprofv3 output dirs: mean duration (kernel trace)
and the mean per dispatch of every PMC counter collected (counter passes).
FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE is also shown x2 in bytes (the
gfx950 correction for 16-B-per-lane streaming reads, MI355X_MICROARCH.md
§HBM). usage: python scripts/pmc_table.py DIR [DIR ...] [--match SUBSTR]"""
import csv
import glob
import os
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
dur = defaultdict(list)
ctr = defaultdict(lambda: defaultdict(list))
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            ctr[k][c].append(v)
names = sorted(set(dur) | set(ctr), key=lambda k: -sum(dur.get(k, [0])))
for k in names:
    if match not in k:
        continue
    short = k.split("(")[0][-90:]
    line = f"{short}\n    n={len(dur.get(k, []))} mean={sum(dur[k]) / len(dur[k]) / 1e3:.2f} us" if k in dur else \
        f"{short}\n    (no trace)"
    for c, v in sorted(ctr.get(k, {}).items()):
        m = sum(v) / len(v)
        line += f"  {c}={m:.4g}"
        if c == "FETCH_SIZE":
            line += f" (x2 bytes={m * 2048:.4g})"
    print(line)
