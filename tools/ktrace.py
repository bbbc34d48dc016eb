"""Per-dispatch summary of a rocprofv3 kernel_trace.csv: kernel, grid, duration (us), in order."""
import csv
import re
import sys

path = sys.argv[1]
lim = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
with open(path) as f:
    rows = list(csv.DictReader(f))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = None
for r in rows[:lim]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\(.*", "", name)[:40]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = t0 or s
    print(f"{(s - t0)/1e3:12.1f} {name:40s} grid {int(r['Grid_Size_X'])//int(r['Workgroup_Size_X']):7d}x{r['Workgroup_Size_X']:>5s} "
          f"{(e - s)/1e3:10.1f} us  vgpr {r['VGPR_Count']} sgpr {r['SGPR_Count']} lds {r['LDS_Block_Size']}")
