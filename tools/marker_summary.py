"""Summary of a rocprofv3 --marker-trace --kernel-trace run of bench.py with AAC_ROCTX=1:
python tools/marker_summary.py DIR [OUT.txt]

Host ranges (roctx: act, env_step, update, update.graph, timed_steps) from run_marker_api_stats.csv,
then the timed region: wall time per step, GPU busy time (union of kernel intervals) and the
kernel time per step by kernel name."""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
    st = list(csv.DictReader(open(os.path.join(d, "run_marker_api_stats.csv"))))
    print("host roctx ranges (enqueue-side durations):", file=out)
    print(f"  {'range':16s} {'calls':>6s} {'avg us':>10s} {'total ms':>10s}", file=out)
    for r in st:
        print(f"  {r['Name']:16s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:10.2f} "
              f"{float(r['TotalDurationNs']) / 1e6:10.3f}", file=out)
    mt = list(csv.DictReader(open(os.path.join(d, "run_marker_api_trace.csv"))))
    kt = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in kt)
    tw = [m for m in mt if m["Function"] == "timed_steps"]
    if not tw:
        return
    t0, t1 = int(tw[0]["Start_Timestamp"]), int(tw[0]["End_Timestamp"])
    steps = sorted((int(m["Start_Timestamp"]), m["Function"]) for m in mt
                   if m["Function"] in ("act", "env_step", "update") and t0 <= int(m["Start_Timestamp"]) <= t1)
    inwin = [k for k in ks if t0 <= k[0] < t1]     # timed_steps ends after its closing synchronize
    n_act = sum(1 for _, f in steps if f == "act")
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in inwin:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    last = max(e for _, e, _ in inwin) if inwin else t1
    wall = last - t0
    print(f"\ntimed region: {n_act} steps, host {(t1 - t0) / 1e6:.3f} ms, host + drain {wall / 1e6:.3f} ms "
          f"({wall / 1e3 / max(n_act, 1):.1f} us per step), {len(inwin)} kernels, GPU busy "
          f"{busy / 1e6:.3f} ms ({100.0 * busy / max(wall, 1):.1f} %)", file=out)
    # the host runs ahead of the GPU (the ranges are enqueue windows), so the kernels are grouped by name
    per = {}
    for s_, e, name in inwin:
        k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        per.setdefault(k, [0, 0])
        per[k][0] += e - s_
        per[k][1] += 1
    print("kernels of the timed region per step (by name):", file=out)
    for k, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0]):
        print(f"  {k[:48]:48s} {n / max(n_act, 1):6.1f} launches {t / 1e3 / max(n_act, 1):9.1f} us", file=out)

if __name__ == "__main__":
    main()
