"""Per-step kernel time of the last K steps of a rocprofv3 kernel trace, steps delimited by a
marker kernel (default the env step kernel): python tools/trace_window.py run_kernel_trace.csv
[K] [marker] [skip].  skip: trailing steps left out -- bench.py runs 10 eager env-timing steps after
a graph-replayed timed region, so the timed steps of configs 3 and 4 are the ones before those."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
marker = sys.argv[3] if len(sys.argv) > 3 else "::step_kernel("
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
skip = int(sys.argv[4]) if len(sys.argv) > 4 else 0
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a, b = idx[-K - 1 - skip], idx[-1 - skip]
seg = rows[a:b]
ksum = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1e3
# GPU busy = the union of the kernel intervals (kernels on two streams overlap)
busy, end = 0, None
for r in seg:
    s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if end is None or s0 >= end:
        busy += e0 - s0
        end = e0
    elif e0 > end:
        busy += e0 - end
        end = e0
busy /= 1e3
wall = (int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
print(f"{'last' if not skip else f'{skip} eager steps skipped, then the last'} {K} steps: {len(seg) / K:.1f} launches/step, kernel time {ksum / K:.1f} us/step, "
      f"wall {wall / K:.1f} us/step (GPU busy {100 * busy / wall:.1f} %"
      + (f", kernels overlapping {ksum - busy:.0f} us over {K} steps)" if ksum > busy + 1 else ")"))
agg = collections.defaultdict(lambda: [0.0, 0])
for r in seg:
    agg[r["Kernel_Name"][:100]][0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 / K
    agg[r["Kernel_Name"][:100]][1] += 1
for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0]):
    print(f"{t:8.1f} us/step {c / K:5.1f} calls/step {t * K / c:7.1f} us/call  {n}")
