"""Per-launch PMC summary of several kernels from rocprofv3 --pmc passes (each pass its own run).

python tools/pmc_kernels.py OUT.json --fetch F.csv --write W.csv --sq S1.csv [--sq S2.csv ...]
                            --kernel NAME=SUBSTR [--kernel ...] [key=value ...]

For each kernel (rows whose Kernel_Name contains SUBSTR) every counter is averaged over its launches
(mean: the launches of one kernel may differ in size, e.g. the attention launches of one update).
HBM bytes per launch follow MI355X_MICROARCH.md: FETCH_SIZE / WRITE_SIZE are KiB, and gfx950's
FETCH_SIZE counts half of a wide coalesced read, so the read side is doubled (raw values kept).
The fp64 VALU counters give fp64_flop_per_launch = 64 (ADD + MUL + 2 FMA + TRANS) (every lane
active: an upper bound).  key=value pairs are copied to the top level (ints where they parse).
"""
import argparse
import collections
import csv
import json
import statistics


def means(paths, sub):
    vals = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            if sub in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: (statistics.fmean(v), len(v)) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--fetch", action="append", default=[])
    ap.add_argument("--write", action="append", default=[])
    ap.add_argument("--sq", action="append", default=[])
    ap.add_argument("--kernel", action="append", required=True)
    ap.add_argument("extra", nargs="*")
    a = ap.parse_intermixed_args()
    res = {}
    for kv in a.extra:
        k, v = kv.split("=", 1)
        try:
            v = int(v)
        except ValueError:
            pass
        res[k] = v
    for spec in a.kernel:
        name, sub = spec.split("=", 1)
        m = means(a.fetch + a.write + a.sq, sub)
        r = {"substr": sub, "launches": {k: n for k, (_, n) in m.items()}}
        for k, (v, _) in m.items():
            r[k] = v
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            f, w = m["FETCH_SIZE"][0], m["WRITE_SIZE"][0]
            r["hbm_bytes_per_launch"] = (2 * f + w) * 1024
            r["hbm_bytes_per_launch_uncorrected"] = (f + w) * 1024
        f64 = [m.get(k, (0.0, 0))[0] for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                                "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")]
        if any(f64):
            r["fp64_insts_per_launch"] = sum(f64)
            r["fp64_flop_per_launch"] = 64.0 * (f64[0] + f64[1] + 2 * f64[2] + f64[3])
        res[name] = r
    res["method"] = ("rocprofv3 --kernel-trace --pmc, one pass per counter group; mean per launch; HBM read "
                     "side x2 (gfx950 FETCH_SIZE half-count)")
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
