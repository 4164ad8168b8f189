"""Per-launch HBM traffic of a kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

MI355X_MICROARCH.md (HBM): both counters are in KiB; on gfx950 FETCH_SIZE reports exactly half of
the bytes of a wide (16 B/lane) coalesced streaming read, so the read side is doubled; WRITE_SIZE
is exact for 16-B stores.  The env state loads are 16-B double2 per lane, so the correction is
applied to the whole fetch (an upper bound for the narrower loads) and the raw value is kept.

python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_SUBSTR ENVS AGENTS RADAR OUT.json
"""
import csv
import json
import statistics
import sys


def per_launch(path, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    return statistics.median(vals[2:] if len(vals) > 4 else vals), len(vals)


def main():
    fpath, wpath, kernel, envs, agents, radar, out = sys.argv[1:8]
    f, nf = per_launch(fpath, "FETCH_SIZE", kernel)
    w, nw = per_launch(wpath, "WRITE_SIZE", kernel)
    N = int(agents)
    alg = (130 + 4 * (24 + 10 * (N - 1))) * int(envs) * N
    res = {"kernel": kernel, "envs": int(envs), "agents": N, "radar": radar,
           "fetch_size_kib_raw": f, "write_size_kib": w, "launches": [nf, nw],
           "hbm_bytes_per_launch": (2 * f + w) * 1024, "hbm_bytes_per_launch_uncorrected": (f + w) * 1024,
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": (2 * f + w) * 1024 / alg,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace; "
                     "median over launches; read side x2 (gfx950 FETCH_SIZE half-count)"}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
