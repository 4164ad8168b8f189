"""Per-launch durations of one training step from a rocprofv3 kernel trace, between two
replay-sample launches: python tools/update_trace.py run_kernel_trace.csv [which].  bench.py ends
with 4 eager updates for the GEMM roofline (CPU launch gaps), so the default window (-6) is the
last graph-replayed step of the timed region."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -6
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
a, b = idx[which - 1], idx[which]
tot = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot += d
    wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
    print(f"{d:8.1f} us {wg:7d} wg  {r['Kernel_Name'][:70]}")
print(f"sum {tot:.1f} us, wall {(int(rows[b]['Start_Timestamp']) - int(rows[a]['Start_Timestamp'])) / 1000:.1f} us")
