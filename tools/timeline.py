"""Per-run kernel timeline from a rocprofv3 --kernel-trace CSV: durations and the idle gaps
between consecutive kernels (all queues merged), averaged over the runs of the F plan.

  python tools/timeline.py <kernel_trace.csv> [first_kernel_substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_f8_solve"
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
                for r in rows)
    runs, cur = [], []
    for e in ev:
        if first in e[2] and cur:
            runs.append(cur)
            cur = []
        cur.append(e)
    runs.append(cur)
    runs = runs[3:-1] if len(runs) > 5 else runs  # drop warm-up and the last partial run
    dur, gap = defaultdict(list), defaultdict(list)
    period = []
    for i, r in enumerate(runs):
        for k, (s, e, n) in enumerate(r):
            dur[(k, n)].append(e - s)
            if k:
                gap[(k, n)].append(s - r[k - 1][1])
        if i + 1 < len(runs):
            period.append(runs[i + 1][0][0] - r[0][0])
    for (k, n), v in sorted(dur.items()):
        g = gap.get((k, n), [0])
        print(f"{k:2d} {n[-40:]:40s} dur {sum(v) / len(v) / 1e3:8.2f} us   gap-before "
              f"{sum(g) / len(g) / 1e3:7.2f} us")
    if period:
        print(f"run period {sum(period) / len(period) / 1e3:.2f} us over {len(period)} runs")


if __name__ == "__main__":
    main()
