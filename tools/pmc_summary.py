"""Per-launch HBM traffic of a kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

MI355X_MICROARCH.md (HBM): both counters are in KiB; on gfx950 FETCH_SIZE reports exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so the read side is doubled; WRITE_SIZE
is exact for 16-B stores.  The correction is applied to the whole fetch (an upper bound for the
narrower loads) and the raw values are kept.

python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR STAT OUT.json [key=value ...]
  STAT     median (one kernel, identical launches) or mean (a kernel whose launches differ, e.g.
           the grouped GEMM: mean HBM bytes per launch over the run)
  key=value  fields copied into the JSON (ints where they parse), e.g. envs=4096 agents=5
             algorithmic_bytes_per_launch=7905280
"""
import csv
import json
import statistics
import sys


def per_launch(path, counter, kernel, stat):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if stat == "mean":
        return statistics.fmean(vals), len(vals)
    return statistics.median(vals[2:] if len(vals) > 4 else vals), len(vals)


def main():
    fpath, wpath, kernel, stat, out = sys.argv[1:6]
    extra = {}
    for kv in sys.argv[6:]:
        k, v = kv.split("=", 1)
        try:
            v = int(v)
        except ValueError:
            pass
        extra[k] = v
    f, nf = per_launch(fpath, "FETCH_SIZE", kernel, stat)
    w, nw = per_launch(wpath, "WRITE_SIZE", kernel, stat)
    res = {"kernel": kernel, **extra, "fetch_size_kib_raw": f, "write_size_kib": w, "launches": [nf, nw],
           "hbm_bytes_per_launch": (2 * f + w) * 1024, "hbm_bytes_per_launch_uncorrected": (f + w) * 1024,
           "method": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace; {stat} "
                     "over launches; read side x2 (gfx950 FETCH_SIZE half-count)"}
    alg = extra.get("algorithmic_bytes_per_launch")
    if alg:
        res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / alg
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
