"""Summarise a rocprofv3 kernel_stats.csv per training step."""
import csv, sys
path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.3f} ms/step over {steps:g} steps)")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r['Name'].replace('(anonymous namespace)::', '')[:90]
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% calls/step={int(r['Calls'])/steps:6.1f} avg_us={float(r['AverageNs'])/1e3:8.1f}  {n}")
