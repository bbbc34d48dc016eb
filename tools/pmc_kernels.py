"""Per-kernel per-launch averages of every PMC counter in rocprofv3 --pmc csv outputs.
  python tools/pmc_kernels.py <dir> [<dir> ...]   (kernels named by their template head)"""
import csv
import glob
import re
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for d in sys.argv[1:]:
    for p in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
            name = re.sub(r"\(.*", "", name)[:48]
            vals[name][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(name, r["Counter_Name"])].add(r["Dispatch_Id"])
for name in sorted(vals):
    print(name)
    for c, v in sorted(vals[name].items()):
        n = len(disp[(name, c)])
        print(f"    {c:26s} {v / max(n, 1):16.4g}  (launches {n})")
