"""Turn the gpurun_out/ results of tools/evidence_round.sh into the committed profiles/ files:
bench lines, per-step kernel summaries (last 5 traced steps), kernel stats, and the PMC traffic
files the bench reads (HBM bytes per launch next to the algorithmic bytes).

python tools/evidence_summary.py bench | pmc  (round tag from AAC_ROUND, default r03)
"""
import csv
import json
import os
import shutil
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT, PROF = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
R = os.environ.get("AAC_ROUND", "r03")


def bench_line(label):
    with open(os.path.join(OUT, label + ".log")) as f:
        lines = [ln for ln in f.read().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def trace_csv(d):
    for root, _, files in os.walk(os.path.join(OUT, d)):
        for fn in files:
            if fn.endswith("kernel_trace.csv"):
                return os.path.join(root, fn)
    raise FileNotFoundError(d)


def stats_csv(d):
    return trace_csv(d).replace("kernel_trace.csv", "kernel_stats.csv")


def counter_csv(d):
    return trace_csv(d).replace("kernel_trace.csv", "counter_collection.csv")


def per_launch(path, counter, kernel, stat):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if stat == "mean":
        return statistics.fmean(vals), len(vals)
    return statistics.median(vals[2:] if len(vals) > 4 else vals), len(vals)


def traffic(fdir, wdir, kernel, stat, extra, out_names):
    f, nf = per_launch(counter_csv(fdir), "FETCH_SIZE", kernel, stat)
    w, nw = per_launch(counter_csv(wdir), "WRITE_SIZE", kernel, stat)
    res = {"kernel": kernel, **extra, "fetch_size_kib_raw": f, "write_size_kib": w, "launches": [nf, nw],
           "hbm_bytes_per_launch": (2 * f + w) * 1024, "hbm_bytes_per_launch_uncorrected": (f + w) * 1024,
           "method": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) --kernel-trace; {stat} over "
                     "launches; read side x2 (gfx950 FETCH_SIZE half-count of 16-B/lane reads, an upper bound for "
                     "narrower reads); uncorrected value kept"}
    alg = extra.get("algorithmic_bytes_per_launch")
    if alg:
        res["traffic_over_algorithmic"] = res["hbm_bytes_per_launch"] / alg
        res["traffic_over_algorithmic_uncorrected"] = res["hbm_bytes_per_launch_uncorrected"] / alg
    for name in out_names:
        with open(os.path.join(PROF, name), "w") as fh:
            json.dump(res, fh, indent=1)
    print(name, json.dumps(res))


def main():
    what = sys.argv[1]
    if what == "bench":
        for label, name in (("bench", f"{R}_bench.json"), ("bench_gru", f"{R}_bench_gru.json"),
                            ("bench_uam", f"{R}_bench_uam.json")):
            d = bench_line(label)
            with open(os.path.join(PROF, name), "w") as fh:
                json.dump(d, fh, indent=1)
            print(name, d["value"], d["ms_per_step"], d["roofline"].get("frac"))
        # configs 3 / 4: the timed steps are graph replays (two steps each), followed by 10 eager
        # env-timing steps, which the window skips; config 5 runs eagerly
        for d, name, marker, k, skip in (("prof3", "train_step", "::step_kernel", "6", "10"),
                                         ("prof4", "gru_step", "::step_kernel", "6", "10"),
                                         ("prof5", "uam_step", "uam_step_kernel", "5", "0")):
            txt = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_window.py"), trace_csv(d), k,
                                  marker, skip], capture_output=True, text=True, check=True).stdout
            with open(os.path.join(PROF, f"{R}_{name}_summary.txt"), "w") as fh:
                fh.write(txt)
            shutil.copy(stats_csv(d), os.path.join(PROF, f"{R}_{name}_kernel_stats.csv"))
            print(txt.splitlines()[0])
    elif what == "pmc":
        b3 = json.load(open(os.path.join(PROF, f"{R}_bench.json")))
        b4 = json.load(open(os.path.join(PROF, f"{R}_bench_gru.json")))
        for b, fd, wd, names, model in ((b3, "pmc3f", "pmc3w", [f"{R}_gemm_pmc.json", "gemm_pmc.json"], "att"),
                                        (b4, "pmc4f", "pmc4w", [f"{R}_gemm_pmc_gru.json", "gemm_pmc_gru.json"], "gru")):
            c, rf = b["config"], b["roofline"]
            traffic(fd, wd, "gemm_kernel", "mean",
                    {"model": model, "envs": c["envs_per_gpu"] if "envs_per_gpu" in c else c.get("envs"),
                     "agents": c.get("agents"), "batch": c.get("batch"),
                     "algorithmic_bytes_per_launch": int(rf["algorithmic_bytes_per_launch"])}, names)
        for b, fd, wd, names, variant, radar in (
                (b3, "pmc3f", "pmc3w", [f"{R}_env_step_pmc.json", "env_step_pmc.json"], "att", "combined"),
                (b4, "pmc4f", "pmc4w", [f"{R}_env_step_pmc_n8.json", "env_step_pmc_n8.json"], "wgru", "obstacles")):
            c, er = b["config"], b["env_roofline"]
            traffic(fd, wd, "::step_kernel", "median",
                    {"envs": c["envs_per_gpu"] if "envs_per_gpu" in c else c.get("envs"), "agents": c.get("agents"),
                     "radar": radar, "variant": variant, "maps": c.get("maps", 1),
                     "tail": "aac_env_step_tail" in er["kernel"],
                     "algorithmic_bytes_per_launch": int(er["bytes_per_agent_step"] * er["agents_per_launch"])},
                    names)
        from bench import env_bytes_per_agent_step     # noqa: E402  (ATT env, N = 5)
        traffic("pmcef", "pmcew", "::step_kernel", "median",
                {"envs": 262144, "agents": 5, "radar": "combined", "variant": "att",
                 "algorithmic_bytes_per_launch": int(env_bytes_per_agent_step(5) * 262144 * 5)},
                [f"{R}_env_step_pmc_262144.json"])
        b5 = json.load(open(os.path.join(PROF, f"{R}_bench_uam.json")))
        c5 = b5["config"]
        traffic("pmc5f", "pmc5w", "uam_step_kernel", "median",
                {"envs": c5["envs_per_gpu"], "agents": c5["agents"], "tdcpa": bool(c5.get("tdcpa")),
                 "algorithmic_bytes_per_launch": int(b5["env_roofline"]["bytes_per_agent_step"] *
                                                     b5["env_roofline"]["agents_per_launch"])},
                [f"{R}_uam_env_pmc.json", "uam_env_pmc.json"])
        shutil.copy(os.path.join(OUT, "gt.log"), os.path.join(PROF, f"{R}_gemm_table.txt"))
        rows = [r for r in csv.DictReader(open(counter_csv("pmcsq"))) if "::step_kernel" in r["Kernel_Name"]]
        by = {}
        for r in rows:
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        sq = {k: statistics.median(v) for k, v in by.items()}
        res = {"kernel": "step_kernel", "envs": 262144, "agents": 5, "radar": "combined",
               "counters_median_per_launch": sq,
               "wait_inst_frac": sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
               "active_inst_frac": sq["SQ_ACTIVE_INST_ANY"] / sq["SQ_WAVE_CYCLES"],
               "wait_any_frac": sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"],
               "note": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_ANY in quad-cycles; GRBM_GUI_ACTIVE summed "
                       "over 8 XCDs; tools/env_only.py --envs 262144 --steps 6, one --pmc pass"}
        with open(os.path.join(PROF, f"{R}_env_sq_262144.json"), "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res))


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    main()
