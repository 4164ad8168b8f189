"""Per-position FETCH_SIZE / WRITE_SIZE of the grouped-GEMM launches of the last traced updates:
python tools/pmc_gemm_pos.py <fetch dir> <write dir> [launches per update]"""
import csv
import os
import sys


def counter_csv(d):
    for root, _, files in os.walk(d):
        for fn in files:
            if fn.endswith("counter_collection.csv"):
                return os.path.join(root, fn)
    raise FileNotFoundError(d)


def vals(d, counter):
    rows = [r for r in csv.DictReader(open(counter_csv(d))) if r["Counter_Name"] == counter and "gemm_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [(r["Kernel_Name"].split("(")[0][-22:], float(r["Counter_Value"])) for r in rows]


f, w = vals(sys.argv[1], "FETCH_SIZE"), vals(sys.argv[2], "WRITE_SIZE")
per = int(sys.argv[3]) if len(sys.argv) > 3 else 8
nup = 5
f, w = f[-per * nup:], w[-per * nup:]
print(f"{'pos':>3} {'kernel':>22} {'fetch KiB':>10} {'write KiB':>10}")
tot = 0
for p in range(per):
    fk = sum(f[p + per * i][1] for i in range(nup)) / nup
    wk = sum(w[p + per * i][1] for i in range(nup)) / nup
    tot += 2 * fk + wk
    print(f"{p:3d} {f[p][0]:>22} {fk:10.1f} {wk:10.1f}")
print(f"mean corrected bytes per launch {tot * 1024 / per:.0f}")
