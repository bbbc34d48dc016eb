"""Per-launch averages of every counter of one kernel in rocprofv3 --pmc csv outputs.
  python tools/pmc_read.py <dir> [kernel-substring]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
k = sys.argv[2] if len(sys.argv) > 2 else "k_f8_count32"
vals = defaultdict(list)
for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if k in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for c, v in sorted(vals.items()):
    print(f"{c:28s} {sum(v)/len(v):16.4g}  (n={len(v)})")
