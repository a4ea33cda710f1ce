"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time (ms per step if --steps)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.1f} ms ({tot / 1e6 / steps:.1f} ms/step over {steps:g} steps)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {int(r['Calls']):6d} calls "
          f"{float(r['AverageNs']) / 1e3:9.1f} us avg {float(r['Percentage']):5.1f}%  {r['Name'][:100]}")
