"""Print the two bench lines and the per-kernel stats (name filter argv[1]) of an A/B run."""
import csv
import json
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else ""
for t in "ab":
    d = json.loads([ln for ln in open(f"gpurun_out/ab_{t}.json") if ln.startswith("{")][-1])
    print(t, round(d["value"] / 1e6, 3), round(d["ms_per_step"], 4))
    for r in csv.DictReader(open(f"gpurun_out/ab_prof_{t}/run_kernel_stats.csv")):
        if pat in r["Name"]:
            print("   ", r["Name"][:50], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2),
                  round(float(r["TotalDurationNs"]) / 1e6, 3))
