"""Print a rocprofv3 kernel_stats.csv compactly: name (shortened), calls, avg us, total ms, %."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print(path)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])
            name = re.sub(r"\(.*", "", name)[:60]
            print(f"  {name:60s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us "
                  f"{float(r['TotalDurationNs'])/1e6:9.2f} ms {float(r['Percentage']):6.2f}%")
