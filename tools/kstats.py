"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:n]:
    print(f"{float(r['Percentage']):6.2f}% {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f}us  {r['Name'][:100]}")
