"""Summarise a rocprofv3 kernel_stats.csv: per-step ms per kernel (pass steps count)."""
import csv, sys
path, steps = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% n={int(r['Calls'])/steps:6.1f}/step avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:80]}")
print(f"total {tot/1e6/steps:.3f} ms/step")
