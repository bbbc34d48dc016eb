"""One C2 parse's kernel timeline from a rocprofv3 kernel trace (the last run in the file):
start / end (us from the run's first jump launch), duration, queue.
  python tools/r05_np_timeline.py <kernel_trace.csv>"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
name = [re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]))[:40]
        for r in rows]
jumps = [i for i, n in enumerate(name) if n.startswith("k_mt_jump")]
s0 = jumps[-3]
t0 = int(rows[s0]["Start_Timestamp"])
for i in range(s0, len(rows)):
    a, b = int(rows[i]["Start_Timestamp"]) - t0, int(rows[i]["End_Timestamp"]) - t0
    print(f"{name[i]:42s} {a / 1e3:8.1f} {b / 1e3:8.1f}  dur {(b - a) / 1e3:7.1f}  q{rows[i]['Queue_Id']}")
