"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time (per-call averages)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n_steps = float(sys.argv[2]) if len(sys.argv) > 2 else None
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms" + (f", {tot / 1e6 / n_steps:.3f} ms per step" if n_steps else ""))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    per = f" {float(r['TotalDurationNs']) / 1e3 / n_steps:8.1f} us/step" if n_steps else ""
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {int(r['Calls']):6d} calls {float(r['AverageNs']) / 1e3:8.1f} us"
          f"{per} {float(r['Percentage']):5.1f}%  {r['Name'][:100]}")
