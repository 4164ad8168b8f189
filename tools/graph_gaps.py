"""Kernel-by-kernel durations and the idle gap before each, over the last two env steps of a
rocprofv3 --kernel-trace run: python tools/graph_gaps.py <dir with *kernel_trace.csv> [marker]
(marker: the kernel-name substring that starts a step, default 'step_kernel<')."""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "step_kernel<"
    path = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    a, b = idx[-3], idx[-1]
    prev, tot_gap = None, 0.0
    for r in rows[a:b + 1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        tot_gap += max(gap, 0.0) if prev else 0.0
        print(f"{(e - s) / 1e3:7.2f} us  gap before {gap:6.2f}  {r['Kernel_Name'][:90]}")
        prev = e
    print(f"idle over the two steps: {tot_gap:.1f} us")


if __name__ == "__main__":
    main()
