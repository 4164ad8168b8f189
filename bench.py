"""Benchmark: agent-env-steps/s (whole node) + MADDPG updates/s, one_model_att, 5 agents x 4096 envs.

One timed *step* = one vectorised training iteration of ATT/main:248-447 on every GPU:
  actor forward + exploration noise for E x N agents      (choose_action, ATT/maddpg:455)
  fused env step: kinematics, radar, obs, ss_reward, done (env.step + ss_reward, ATT/env:2627/:2105)
  replay push of E transitions                             (memory.push, ATT/main:400)
  GPU auto-reset of finished envs from the OD bank         (reset_world, ATT/env:199)
  one update_myown-equivalent: N=5 gradient iterations at B=1024 + Polyak (ATT/maddpg:219-440)
value = E_total * N * steps / max-over-ranks wall time.  Inputs are synthetic (seeded map, OD
bank, random-init networks); the replay is pre-filled to 1e5 transitions before timing.

python bench.py [--gpus N] [--steps K] [--warmup W]
N > 1: one process per GPU under torch.distributed.run (RCCL).  When WORLD_SIZE is already set (the
driver's ``torch.distributed.run ... bench.py --gpus N``) this process is one rank; otherwise this
process starts the N ranks itself as a child ``torch.distributed.run`` (before touching the GPU),
waits, and exits with its return code (rank 0 prints the line).

``--model gru`` measures config 4 instead (randomOD_gru_radar): the
same vectorised loop with the GRU-actor MADDPG of MADDPG_ownENV_randomOD_Wgru_radar (one GRU actor
and one GRU critic per agent, hidden states carried per agent, zeroed when an episode ends, and
stored in the replay), 8 agents, B = 512 (its argparse default).  ``--model uam`` measures config 5
(MADDPG_ownENV_randomOD_radar_N_model_use_tdCPA_forV2_changeskin_UAM): the UAM
env kernel (clouds, go-around aircraft, runway, sorted neighbours) with its float64 shared actor /
single critic learner, 16 aircraft x 8192 envs, one gradient iteration per update at B = 512, one
replay row per aircraft.  The default line is config 3.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multi_agent_aac_amd import trace  # noqa: E402  (roctx ranges, off unless AAC_ROCTX=1)

METRIC = "agent-env-steps/sec (whole node) + MADDPG updates/sec, 5 agents×4096 envs"
METRIC_GRU = "agent-env-steps/sec (whole node) + MADDPG updates/sec, 8 agents×4096 envs, GRU actor"
METRIC_UAM = "agent-env-steps/sec (whole node) + MADDPG updates/sec, 16 agents×8192 envs, UAM"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_PEAK_TFLOPS = 157.3
FP64_PEAK_TFLOPS = 78.6    # AMD MI355X spec sheet, dense FP64 vector / matrix (the guide lists no FP64 row)


def env_bytes_per_agent_step(N, variant="att", mean_wp=None):
    """130 + 4 (24 + 10 (N - 1)) algorithmic HBM bytes per agent-env-step.
    WGRU variant (config 4): read pos, vel (32), action (8), goal (16), path start (16), the goal list
    (16 per waypoint, mean_wp of them), removed-bits + count (8); write pos, vel, pre_pos (48); obs
    own 6 + radar 18 + nei 6 (N - 1) floats; reward, done, mask (6)."""
    if variant == "wgru":
        return 80 + 16 * mean_wp + 48 + 4 * (24 + 6 * (N - 1)) + 6
    return 130 + 4 * (24 + 10 * (N - 1))


def push_read_floats(replay):
    """Floats of one transition row the fused tail reads from memory: s_own, s_radar, s_nei, act
    (fields 0-3) and the hidden states h_cur / h_next (fields 9-10); fields 4-8 are this step's
    own outputs, written to the ring without a read-back."""
    w = replay.widths
    return sum(w[:4]) + sum(w[9:])


def env_fp64_flop_per_agent_step(N):
    """~780 (N - 1) + 300 fp64 FLOP per agent-env-step (18 rays x (N - 1)
    64-gon clip windows + kinematics, predicates, reward)."""
    return 780 * (N - 1) + 300


def uam_bytes_per_agent_step(N, tdcpa=True):
    """Algorithmic HBM bytes of one UAM agent-env-step (aac_uam.hip): read
    pos, vel, action, goal, start (5 x 16), heading (8), reach (1), top2 (2) = 91; write pos, vel,
    pre_pos, pre_vel (64), heading (8), reach (1), top2 (2) = 75; float64 observations own 7, radar
    18, neighbours 5 (N - 1); reward 8, done 1, mask 1; with tdCPA live: float64 tcpa and dcpa per
    neighbour, int32 conf_cur and conf_pre."""
    return 91 + 75 + 8 * (7 + 18 + 5 * (N - 1)) + 10 + ((16 * (N - 1) + 8) if tdcpa else 0)


def uam_update_flops(B):
    """2 M N K over the UAM learner's products per update_myown (one gradient iteration at B rows):
    target actor + target critic forward, critic forward + backward (3x), actor forward, critic
    forward on the policy action + backward to the action, actor backward."""
    A = 7 * 64 + 18 * 64 + 128 * 128 + 128 * 2
    C = 9 * 64 + 18 * 64 + 128 * 256 + 256
    return 2.0 * B * (A + C + 3 * C + A + 3 * C + 3 * A)


def update_flops(N, D0, B):
    """(4A + 7C) MACs per sample per gradient iteration, N iterations."""
    K = N - 1
    A = N * (D0 * 64 + 18 * 64 + K * 6 * 64 + 64 * 64 + K * 2 * 64 * 64 + 192 * 256 + 256 * 2)
    C = N * (D0 + 2) * 128 + 128 * N * 256 + 256
    return 2.0 * (4 * A + 7 * C) * B * N


def gemm_roofline(model, B, reps=10):
    """Roofline of the dominant kernel, the grouped fp32 MFMA GEMM (gemm_kernel) of the fused
    learner, after the timed region: one eager update_myown-equivalent, then every grouped-GEMM
    launch of it replayed ``reps`` times back to back from a captured HIP graph between a HIP event
    pair on the replay stream -- the launch's device duration without host launch gaps, as the
    rocprof kernel trace reports it (profiles/).  achieved = algorithmic FLOPs of the launches /
    the sum of their durations."""
    from multi_agent_aac_amd.fused import GemmLaunch
    flops, us, nbytes, n = time_launches(model, B, (GemmLaunch,), reps)
    achieved = flops / (us * 1e-6) / 1e12
    return {"kernel": "gemm_kernel (grouped fp32 MFMA GEMM of the fused learner)", "bound": "mfma",
            "achieved": achieved, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP32_PEAK_TFLOPS,
            "flop_per_launch": flops / n, "algorithmic_bytes_per_launch": nbytes / n,
            "avg_launch_ms": us / n / 1e3, "launches_per_update": n,
            "gemm_ms_per_update": us / 1e3, "timing": f"graph replay x{reps} per launch, HIP events"}


def time_launches(model, B, kinds, reps=10):
    """One eager update_myown-equivalent, then every launch of it whose type is in ``kinds`` replayed
    ``reps`` times back to back from a captured HIP graph between a HIP event pair on the replay stream
    (the launch's device duration without host gaps, as in the rocprof kernel trace).  Returns (sum of
    their algorithmic FLOPs, sum of their durations in us, sum of algorithmic bytes, launch count)."""
    fu = model._fused_plan(B) if hasattr(model, "_fused_plan") else model._plan(B)
    ops = fu.ops()
    for op in ops:
        op()
    torch.cuda.synchronize()
    flops, us, nbytes, n = 0.0, 0.0, 0.0, 0
    for op in ops:
        if not isinstance(op, kinds):
            continue
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                op()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        us += e0.elapsed_time(e1) / reps * 1e3
        flops += op.flops
        nbytes += op.bytes
        n += 1
    return flops, us, nbytes, n


def attn_roofline(model, B, reps=10, traffic_file=None):
    """The actor's attention kernels of the fused learner (ActorNetwork_ATT_TwoPortion, ATT/nets:194-213)
    against the fp32 MFMA peak: attn_enc_kernel (encoders + attention forward, riding critic encoders
    and head jobs; fused.attn_enc_cost) and attn_mfma_bwd_kernel (fused.AttnBwd), timed per launch as
    the GEMM roofline.  With a committed PMC file for this config, the HBM traffic per launch."""
    from multi_agent_aac_amd.fused import AttnBwd, AttnEnc
    pm = {}
    if traffic_file and os.path.exists(traffic_file):
        with open(traffic_file) as f:
            pm = json.load(f)
    out = {}
    for name, kind in (("attn_enc_kernel", AttnEnc), ("attn_mfma_bwd_kernel", AttnBwd)):
        flops, us, nbytes, n = time_launches(model, B, (kind,), reps)
        if not n:
            continue
        ach = flops / (us * 1e-6) / 1e12
        r = {"bound": "mfma", "achieved": ach, "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
             "frac": ach / FP32_PEAK_TFLOPS, "flop_per_launch": flops / n, "algorithmic_bytes_per_launch": nbytes / n,
             "avg_launch_ms": us / n / 1e3, "launches_per_update": n, "ms_per_update": us / 1e3,
             "hbm_frac_of_algorithmic_bytes": nbytes / (us * 1e-6) / 1e9 / HBM_PEAK_GBS}
        k = pm.get(name)
        if k:
            r["traffic"] = k.get("hbm_bytes_per_launch")
            r["traffic_over_algorithmic"] = r["traffic"] / r["algorithmic_bytes_per_launch"]
            r["pmc"] = {x: k[x] for x in k if x.startswith("SQ_")}
            r["traffic_source"] = os.path.relpath(traffic_file, ROOT)
        out[name] = r
    return out


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--model", default="att", choices=["att", "gru", "uam"],
                   help="att: config 3 (default); gru: config 4, GRU actor (defaults 8 agents, B=512); "
                        "uam: config 5 (16 aircraft x 8192 envs, B=512)")
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--envs", type=int, default=None, help="envs per GPU (default 4096; uam 8192)")
    p.add_argument("--agents", type=int, default=None, help="default 5 (att) / 8 (gru)")
    p.add_argument("--batch", type=int, default=None, help="default 1024 (att) / 512 (gru)")
    p.add_argument("--memory", type=int, default=None, help="replay rows (default 1e5; uam 2^20)")
    p.add_argument("--radar", default="combined", choices=["drones", "obstacles", "combined"])
    p.add_argument("--maps", type=int, default=1,
                   help="att / gru: a stack of this many synthetic maps (seeds 2026..), one drawn per env "
                        "episode (the multipleMap variant, multipleMap/ma_main:464-465)")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-procs", type=int, default=None,
                   help="CPU-baseline processes (default: physical cores, capped at the GPU box's per-GPU CPU "
                        "share of 16, AAC_CPU_SHARE)")
    p.add_argument("--launch-check", action="store_true",
                   help="N > 1 plumbing check: every rank joins the process group (gloo), prints its rank and "
                        "exits without touching the GPU")
    p.add_argument("--cpu-seconds", type=float, default=15.0)
    p.add_argument("--no-seg-overhead", dest="seg_overhead", action="store_false",
                   help="skip the one-GPU timing of the world > 1 update schedule (tools/seg_overhead.py)")
    p.add_argument("--env-micro", type=int, default=1 << 18, help="envs for the env-only HBM microbench (0 = skip)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "env_step_pmc.json"))
    p.add_argument("--gemm-traffic", default=None,
                   help="GEMM PMC file (default profiles/gemm_pmc.json; config 4: profiles/gemm_pmc_gru.json)")
    a = p.parse_args()
    if a.agents is None:
        a.agents = {"gru": 8, "uam": 16}.get(a.model, 5)
    if a.batch is None:
        a.batch = 1024 if a.model == "att" else 512
    if a.envs is None:
        a.envs = 8192 if a.model == "uam" else 4096
    if a.memory is None:
        a.memory = (1 << 20) if a.model == "uam" else 100000
    if a.gemm_traffic is None:
        a.gemm_traffic = os.path.join(ROOT, "profiles", "gemm_pmc_gru.json" if a.model == "gru" else "gemm_pmc.json")
    return a


def launch_ranks(a, argv):
    """``--gpus N`` (N > 1) outside a torch.distributed.run environment: start the N ranks as a child
    ``python -m torch.distributed.run --standalone --local-addr 127.0.0.1 --nproc-per-node N`` of this
    script (one process per GPU, RCCL), before anything here has touched the GPU (no exec: a child
    process).  ``--standalone`` lets the c10d rendezvous bind its own free port (no probe-then-bind
    race with other processes on a shared host).  The CPU baseline is a 1-GPU field (rank 0 at N = 1
    only), so the ranks skip it.  Returns the child's exit code; rank 0's JSON line reaches stdout
    directly."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
           f"--nproc-per-node={a.gpus}", os.path.abspath(__file__)] + list(argv)
    if "--no-cpu-baseline" not in argv:
        cmd.append("--no-cpu-baseline")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC only on this host driver (RCCL)
    return subprocess.run(cmd, env=env).returncode


def setup_dist(backend):
    from multi_agent_aac_amd import parallel
    ws, rank, local, _ = parallel.init_from_env(backend)
    return ws, rank, local


def barrier(ws):
    if ws > 1:
        dist.barrier()
    torch.cuda.synchronize()


from multi_agent_aac_amd import parallel  # noqa: E402
from multi_agent_aac_amd import trainer as _trainer  # noqa: E402
from multi_agent_aac_amd.trainer import Trainer, UamTrainer  # noqa: E402,F401  (the vectorised ma_main loops)


def cpu_baseline_uam(E, N, B, seconds, procs_req=None):
    """UAM: the reference-shaped scalar oracle env step (oracle/uam_ref.py) on the host cores plus the
    CPU float64 update_myown restatement (bounded sample)."""
    import multiprocessing as mp
    from oracle import uam_learner_ref as R
    procs, phys, cores = baseline_procs(procs_req)
    ctx = mp.get_context("spawn")
    budget = seconds / 2
    with ctx.Pool(procs) as pool:
        res = pool.starmap(_cpu_uam_worker, [(N, budget, w) for w in range(procs)])
    steps = sum(r[0] for r in res)
    env_rate = sum(r[0] / r[1] for r in res) * N                 # agent-env-steps/s over all workers
    one = _cpu_uam_worker(N, budget / 4, 0)                       # one process alone: the scaling ratio
    rate1 = one[0] / one[1] * N
    torch.set_num_threads(procs)
    a, c = R.RefActor().double(), R.RefCritic().double()
    at, ct = R.RefActor().double(), R.RefCritic().double()
    oa, oc = torch.optim.Adam(a.parameters(), lr=1e-4), torch.optim.Adam(c.parameters(), lr=1e-4)
    g = torch.Generator().manual_seed(0)
    b = {k: torch.rand(B, w, generator=g, dtype=torch.float64) for k, w in
         (("own", 7), ("radar", 18), ("act", 2), ("n_own", 7), ("n_radar", 18))}
    b["rew"], b["done"] = torch.rand(B, generator=g, dtype=torch.float64), torch.zeros(B, dtype=torch.float64)
    t0 = time.perf_counter()
    n_upd = 0
    while time.perf_counter() - t0 < budget or n_upd == 0:
        R.ref_update(a, c, at, ct, oa, oc, b)
        n_upd += 1
    t_upd = (time.perf_counter() - t0) / n_upd
    t_iter = E * N / env_rate + t_upd
    return {"value": E * N / t_iter, "unit": "agent-env-steps/s", "cores": procs, "kind": "port",
            "physical_cores": phys, "affinity_cores": cores, "cpu_model": cpu_model(),
            "per_physical_core_extrapolated": _extrapolate(env_rate, procs, phys, t_upd, E, N,
                                                           eff=(env_rate / procs) / rate1),
            "scalar_env_rate_per_process": {"1_process": rate1, f"{procs}_processes": env_rate / procs},
            "sample": (f"reference-shaped scalar UAM env oracle on {procs} processes x 1 env x {N} aircraft, "
                       f"{steps} env steps ({env_rate:.3g} agent-env-steps/s env-only) + CPU float64 "
                       f"update_myown restatement B={B} x {n_upd} ({t_upd * 1e3:.2f} ms each), {procs} threads; "
                       f"value = {E}x{N} agent-steps / (env step + update) per iteration"),
            "env_only": env_rate, "update_ms": t_upd * 1e3}


def _cpu_uam_worker(N, budget, wid):
    import random as _random
    sys.path.insert(0, ROOT)
    from oracle import uam_ref as U
    py, npr = _random.Random(wid), np.random.RandomState(wid)
    env = U.UAMEnv(N)
    env.reset(*U.sample_episode(N, py, npr))
    rng = np.random.default_rng(wid)
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < budget or steps < 2:
        *_, over = env.full_step(rng.uniform(-1, 1, (N, 2)))
        if over:
            env.reset(*U.sample_episode(N, py, npr))
        steps += 1
    return steps, time.perf_counter() - t0


def host_cores():
    """(physical cores = lscpu 'Core(s) per socket' x 'Socket(s)', CPUs in this process's affinity)."""
    import subprocess
    aff = len(os.sched_getaffinity(0))
    per, sockets = None, None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Core(s) per socket:"):
                per = int(line.split(":", 1)[1])
            elif line.startswith("Socket(s):"):
                sockets = int(line.split(":", 1)[1])
    except Exception:
        pass
    return (per * sockets if per and sockets else aff), aff


def baseline_procs(requested=None):
    """Processes of the CPU baseline: one per physical core, capped by the affinity and
    by the GPU box's CPU share per GPU (16, AAC_CPU_SHARE): the host is shared by the jobs of its 8
    GPUs.  Returns (procs, physical cores, affinity CPUs)."""
    phys, aff = host_cores()
    if requested:
        return int(requested), phys, aff
    return max(1, min(phys, aff, int(os.environ.get("AAC_CPU_SHARE", "16")))), phys, aff


def _extrapolate(env_rate, procs, phys, t_upd, E, N, eff=1.0):
    """The same iteration with the env spread over one process per physical core: the measured
    per-process env rate at ``procs`` processes x physical cores, times ``eff`` = the measured
    per-process rate at ``procs`` over the rate of one process alone (the decline from 1 to ``procs``
    processes applied once more from ``procs`` to ``phys``: the host does not scale linearly, BENCH_r05
    212.7 vs 186.7 per process), plus the measured update time.  An extrapolation, not a measurement:
    the pool caps a job at 16 worker processes."""
    eff = min(1.0, eff) if eff and eff > 0 else 1.0
    rate = env_rate / procs * phys * (eff if phys > procs else 1.0)
    return {"value": E * N / (E * N / rate + t_upd), "env_only": rate, "cores": phys, "scaling_factor": eff,
            "basis": (f"measured per-process env rate at {procs} processes x {phys} physical cores x {eff:.3f} "
                      f"(the measured 1 -> {procs}-process per-process ratio) + measured update time")}


def cpu_model():
    """The host CPU model line (lscpu 'Model name'), for the baseline's core-count context."""
    import subprocess
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return "unknown"


def _cpu_update_time(N, B, budget, model, threads):
    """Seconds per update_myown of the torch-CPU restatement (oracle/learner_ref.py or gru_ref.py)."""
    from oracle import learner_ref  # noqa: F401  (checker / baseline only)
    torch.set_num_threads(threads)
    D0 = 6 + 4 * (N - 1)
    if model == "gru":
        from oracle import gru_ref
        import copy
        acts = [gru_ref.RefGRUActor([6, 18, 6], 2) for _ in range(N)]
        crits = [gru_ref.RefGRUCritic([6, 18, 6], 2) for _ in range(N)]
        acts_t, crits_t = copy.deepcopy(acts), copy.deepcopy(crits)
        tr = gru_ref.random_gru_transitions(B, N, 0)
        tr["done"] = tr["done"].float()
        step = lambda o: gru_ref.ref_gru_update(acts, crits, acts_t, crits_t, tr, 6, opts=o)[1]  # noqa: E731
    else:
        actor, critic = learner_ref.RefActor([D0, 18, 6], 2), learner_ref.RefCritic([D0, 18, 6], N, 2)
        actor_t, critic_t = learner_ref.RefActor([D0, 18, 6], 2), learner_ref.RefCritic([D0, 18, 6], N, 2)
        tr = learner_ref.random_transitions(B, N, 0)
        tr["done"] = tr["done"].float()
        step = lambda o: learner_ref.ref_update(actor, critic, actor_t, critic_t, [tr] * N, opts=o)[1]  # noqa: E731
    t0 = time.perf_counter()
    n_upd, opts = 0, None
    while time.perf_counter() - t0 < budget or n_upd == 0:
        opts = step(opts)
        n_upd += 1
    return (time.perf_counter() - t0) / n_upd, n_upd


def cpu_baseline(E, N, B, radar, seconds, model="att", procs_req=None):
    """BASELINE.md's CPU baseline on the host cores (bounded sample of the same workload): the env
    step timed in three forms, each combined with the torch-CPU update_myown restatement as one
    training iteration (value = E x N agent-steps / (env step + update)):
      mode 1  reference-shaped scalar Python (oracle/env_ref.py, ATT/env's per-agent loops), one
              process per core, each on its own envs  -- the headline ``value``
      mode 2  vectorised NumPy over envs (oracle/env_np.py), one process, and one process per core
      C port  the batched C restatement (oracle/aac_oracle.c), one process per core
    Each env rate is agent-env-steps/s summed over the processes (envs are independent)."""
    import multiprocessing as mp
    if model == "uam":
        return cpu_baseline_uam(E, N, B, seconds, procs_req)
    procs, phys, cores = baseline_procs(procs_req)
    ctx = mp.get_context("spawn")
    per = max(1, E // procs)
    slot = seconds / 5
    # config 4 times the randomOD_Wgru_radar env (obstacle radar, WGRU reward), as the GPU line
    variant = "wgru" if model == "gru" else "att"
    if variant == "wgru":
        radar = "obstacles"
    with ctx.Pool(procs) as pool:
        m1 = pool.starmap(_cpu_scalar_worker, [(N, radar, slot, w, variant) for w in range(procs)])
        m2 = pool.starmap(_cpu_numpy_worker, [(min(per, 256), N, radar, slot, w, variant) for w in range(procs)])
        cp = pool.starmap(_cpu_env_worker, [(per, N, radar, slot, w, variant) for w in range(procs)])
    m2_one = _cpu_numpy_worker(min(E, 512), N, radar, slot / 2, 0, variant)
    # one process alone: with the per-process rate of the pool, shows how the scalar env scales with
    # processes (the basis of the per-physical-core extrapolation; the box gives each GPU a 16-CPU
    # share, so no pool of one process per physical core is started there)
    m1_one = _cpu_scalar_worker(N, radar, slot / 2, 0, variant)
    t_upd, n_upd = _cpu_update_time(N, B, slot, model, procs)

    def mode(res, what):
        rate = sum(envs * N * steps / sec for steps, sec, envs in res)
        t_iter = E * N / rate + t_upd
        return {"value": E * N / t_iter, "env_only": rate, "processes": len(res), "what": what}

    sref = "oracle/wgru_env_ref.py" if variant == "wgru" else "oracle/env_ref.py"
    modes = {"scalar_per_core": mode(m1, f"{sref} reference-shaped per-agent Python loop"),
             "scalar_1proc": mode([m1_one], f"{sref} reference-shaped per-agent Python loop, one process"),
             "numpy_1proc": mode([m2_one], "oracle/env_np.py vectorised over envs, one process"),
             "numpy_per_core": mode(m2, "oracle/env_np.py vectorised over envs, one process per core"),
             "c_port_per_core": mode(cp, "oracle/aac_oracle.c batched C restatement, one process per core")}
    head = modes["scalar_per_core"]
    per_proc = {"1_process": modes["scalar_1proc"]["env_only"], f"{procs}_processes": head["env_only"] / procs}
    return {"value": head["value"], "unit": "agent-env-steps/s", "cores": procs, "kind": "port",
            "physical_cores": phys, "affinity_cores": cores, "cpu_model": cpu_model(),
            "per_physical_core_extrapolated": _extrapolate(head["env_only"], procs, phys, t_upd, E, N,
                                                           eff=(head["env_only"] / procs) / modes["scalar_1proc"]["env_only"]),
            "sample": (f"mode 1: reference-shaped scalar env ({sref}, {radar} radar) on {procs} processes "
                       f"x 1 env x {N} agents, {sum(r[0] for r in m1)} env steps in ~{slot:.1f} s "
                       f"({head['env_only']:.3g} agent-env-steps/s env-only) + torch-CPU update_myown restatement "
                       f"B={B} x {n_upd} ({t_upd * 1e3:.1f} ms each, {procs} threads); value = {E}x{N} agent-steps / "
                       f"(env step + update) per iteration; other modes in 'modes'"),
            "env_only": head["env_only"], "update_ms": t_upd * 1e3, "modes": modes,
            "scalar_env_rate_per_process": per_proc}


def _cpu_scalar_worker(N, radar, budget, wid, variant="att"):
    """Mode 1: one reference-shaped ScalarEnv (per-agent Python, oracle/env_ref.py, or
    oracle/wgru_env_ref.py for config 4), random actions, re-drawn OD on episode end; returns
    (env steps, seconds, envs)."""
    sys.path.insert(0, ROOT)
    from multi_agent_aac_amd import world
    from oracle import env_ref, wgru_env_ref
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=1024, seed=wid, max_wp=32)
    rng = np.random.default_rng(wid)
    if variant == "wgru":
        env = wgru_env_ref.WgruEnv(N, occ)
    else:
        env = env_ref.ScalarEnv(N, occ, radar_mode={"drones": 0, "obstacles": 1, "combined": 2}[radar])

    def reset():
        st, wps, cnt = bank.sample_env_od(1, N, rng)
        env.reset([tuple(st[0, i]) for i in range(N)], [[list(w) for w in wps[0, i, :cnt[0, i]]] for i in range(N)])
    reset()
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < budget or steps < 2:
        *_, over = env.full_step(rng.uniform(-1, 1, (N, 2)).astype(np.float32))
        if over:
            reset()
        steps += 1
    return steps, time.perf_counter() - t0, 1


def _cpu_numpy_worker(E, N, radar, budget, wid, variant="att"):
    """Mode 2: E envs of the vectorised NumPy env (oracle/env_np.py) with auto-reset."""
    sys.path.insert(0, ROOT)
    from multi_agent_aac_amd import world
    from oracle import env_np
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=4096, seed=wid, max_wp=32)
    rng = np.random.default_rng(wid)
    env = env_np.NumpyEnv(E, N, occ, W=32, radar_mode={"drones": 0, "obstacles": 1, "combined": 2}[radar],
                          variant=variant)
    st, wps, cnt = bank.sample_env_od(E, N, rng)
    env.reset(st, wps, cnt)
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < budget or steps < 1:
        out = env.step(rng.uniform(-1, 1, (E, N, 2)).astype(np.float32))
        done = out[6].astype(bool)
        if done.any():
            env.reset(st, wps, cnt, env_mask=done)
        steps += 1
    return steps, time.perf_counter() - t0, E


def _cpu_env_worker(E, N, radar, budget, wid, variant="att"):
    sys.path.insert(0, ROOT)
    from multi_agent_aac_amd import world
    from oracle import c_oracle
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=4096, seed=wid, max_wp=32)
    rng = np.random.default_rng(wid)
    mode = {"drones": 0, "obstacles": 1, "combined": 2}[radar]
    co = c_oracle.BatchedOracle(E, N, occ, W=32, radar_mode=mode, variant=variant)
    st, wps, cnt = bank.sample_env_od(E, N, rng)
    co.reset(st, wps, cnt)
    acts = rng.uniform(-1, 1, size=(8, E, N, 2)).astype(np.float32)
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < budget or steps < 2:
        co.step(acts[steps % 8])
        done = co.env_done.astype(bool)
        if done.any():
            co.reset(st, wps, cnt, env_mask=done.astype(np.uint8))
        steps += 1
    return steps, time.perf_counter() - t0, E


def world_schedule_overhead(N, B, updates=20):
    """The world > 1 update schedule's cost per update on this one GPU: the
    N + 1 gradient all-reduces captured in the update graph over a one-rank RCCL group, against the
    world = 1 graph, and the eager segmented alternative (tools/seg_overhead.py, a child process: it
    initialises its own process group).  The 1 -> 8 GPU curve itself is the driver's run."""
    import socket
    import subprocess
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "seg_overhead.py"), "--updates", str(updates),
                            "--agents", str(N), "--batch", str(B)], capture_output=True, text=True, timeout=240,
                           env=env)
        if r.returncode != 0:
            return {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
        res = json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as e:       # reported, never fatal to the bench line
        return {"error": f"{type(e).__name__}: {e}"[:300]}
    res["note"] = ("one GPU, one-rank RCCL group, world = 2 schedule: per-update overhead vs the world = 1 "
                   "graph; segmented_overhead_us is the default (collectives captured in the graph)")
    return res


def env_microbench(E, N, radar, iters=20, variant="att"):
    """Env-only kernel throughput at large E (the HBM-roofline regime of SURVEY 8(d))."""
    from multi_agent_aac_amd import world
    from multi_agent_aac_amd.env import BatchedEnv
    occ = world.synthetic_map(2026)
    bank = world.ODBank(occ, n_pairs=65536, seed=5, max_wp=32)
    env = BatchedEnv(E, N, occ, radar_mode=None if variant == "wgru" else radar, max_wp=32, variant=variant)
    env.set_od_bank(bank, seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(E, N, 2, device="cuda", generator=g) * 2 - 1 for _ in range(4)]
    for i in range(3):
        env.step(acts[i % 4])
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for i in range(iters):
        ev[i][0].record()
        env.step(acts[i % 4])
        ev[i][1].record()
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    rate = E * N / (ms * 1e-3)
    gbs = env_bytes_per_agent_step(N, variant, float(np.mean(bank.cnt))) * E * N / (ms * 1e-3) / 1e9
    return {"envs": E, "agents": N, "variant": variant, "kernel_ms": ms, "agent_env_steps_per_s": rate,
            "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}


def uam_env_microbench(E, N, iters=10):
    """UAM env-only kernel throughput at large E."""
    from multi_agent_aac_amd import uam
    env = uam.BatchedUAM(E, N)
    env.set_bank(uam.build_bank(8192, N, seed=5), seed=3)
    env.auto_reset(None)
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(E, N, 2, device="cuda", generator=g, dtype=torch.float64) * 2 - 1 for _ in range(4)]
    for i in range(3):
        env.step(acts[i % 4])
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for i in range(iters):
        ev[i][0].record()
        env.step(acts[i % 4])
        ev[i][1].record()
        env.auto_reset(env.bufs.env_done)
    torch.cuda.synchronize()
    ms = float(np.mean([x.elapsed_time(y) for x, y in ev]))
    gbs = uam_bytes_per_agent_step(N, tdcpa=False) * E * N / (ms * 1e-3) / 1e9
    return {"envs": E, "agents": N, "kernel_ms": ms, "agent_env_steps_per_s": E * N / (ms * 1e-3),
            "achieved_GBs": gbs, "frac": gbs / HBM_PEAK_GBS}


def main():
    a = parse()
    _trainer.NO_GRAPH = a.no_graph
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, sys.argv[1:]))
    ws0 = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and ws0 != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={ws0}")
    if a.launch_check:
        from multi_agent_aac_amd import parallel
        ws, rank, _, _ = parallel.init_from_env("gloo") if ws0 > 1 else (1, 0, 0, None)
        if ws > 1:
            dist.barrier()
        print(json.dumps({"launch_check": True, "rank": rank, "world_size": ws, "gpus": a.gpus}), flush=True)
        if ws > 1:
            dist.destroy_process_group()
        return
    cpu = None
    if ws0 == 1 and not a.no_cpu_baseline:
        # before any GPU initialisation: the pool's children must not inherit a GPU context
        cpu = cpu_baseline(a.envs, a.agents, a.batch, a.radar, a.cpu_seconds, model=a.model, procs_req=a.cpu_procs)
    ws, rank, local = setup_dist(a.backend)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(777 + rank)
    pg = dist.group.WORLD if ws > 1 else None
    if a.model == "uam":
        tr = UamTrainer(a.envs, a.agents, a.batch, a.memory, seed=rank, pg=pg)
    else:
        tr = Trainer(a.envs, a.agents, a.batch, a.memory, a.radar, seed=rank, pg=pg, model=a.model, maps=a.maps)
    # pre-fill the replay to >= memory transitions (untimed), then capture the update graph
    while len(tr.replay) < min(a.memory, 100000):
        tr.step(update=False)
    for _ in range(a.warmup):
        tr.step(update=True)
    barrier(ws)
    tr.env_events.clear()
    t0 = time.perf_counter()
    graphed = hasattr(tr, "graph_ok") and tr.graph_ok()
    # several steps per graph replay (the buffer parities in sequence: fewer graph-launch gaps): the
    # largest of AAC_STEP_GROUP (default 2: 4 measured slower, profiles/r06_step_group_ab.txt) and 2 that
    # divides the step count; AAC_STEP_PAIR=0 replays
    # one step per graph
    group = 1
    if graphed and os.environ.get("AAC_STEP_PAIR", "1") == "1":
        group = next((g for g in (int(os.environ.get("AAC_STEP_GROUP", "2")), 2) if g >= 2 and g % 2 == 0
                      and a.steps % g == 0), 1)
    pairs = group > 1
    if graphed:
        for _ in range(2):        # capture (untimed) and replay once
            if pairs:
                tr.step_graph_pair(group)
            else:
                tr.step_graph()
        torch.cuda.synchronize()
        barrier(ws)
        t0 = time.perf_counter()
    with trace.range("timed_steps"):
        for k in range(a.steps // group):
            if pairs:
                tr.step_graph_pair(group)
            elif graphed:
                tr.step_graph()
            else:
                # HIP events around the env launch on every 5th timed step only: an event pair costs
                # ~5 us of stream time on each side of the launch it brackets
                tr.step(update=True, time_env=(k % 5 == 0))
    barrier(ws)
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], device="cuda")
    if ws > 1:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t)
    if graphed:
        # the env launch is inside the step graphs: time it on 10 eager steps after the timed region
        for k in range(10):
            tr.step(update=True, time_env=True)
        torch.cuda.synchronize()
    env_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in tr.env_events]))
    # the exact threshold fix-up list never overflowed in this run (else the surplus rays kept their float
    # decisions): checked once, after the timed region (synchronises)
    band = None if a.model == "uam" else tr.env.check_band_capacity()
    E_total = a.envs * ws
    N = a.agents
    value = E_total * N * a.steps / dt
    upd_per_s = a.steps / dt
    uam = a.model == "uam"
    D0 = 6 + 4 * (N - 1)
    if uam:
        bpa = uam_bytes_per_agent_step(N)
    elif tr.gru:
        bpa = env_bytes_per_agent_step(N, "wgru", float(np.mean(tr.bank.cnt)))
    else:
        bpa = env_bytes_per_agent_step(N)
    push_bpa = 0.0
    if not uam and tr.fused_tail:
        # the fused tail's replay push: every ring row is written once; the fields this step produces
        # (reward, done, next own / radar / nei) go to the ring from the kernel's registers / LDS, so
        # only the carried-in fields (current obs rows, actions, hidden states) are read
        push_bpa = 4.0 * (tr.replay.row_width + push_read_floats(tr.replay)) / N
        bpa += push_bpa
    achieved = bpa * a.envs * N / (env_ms * 1e-3) / 1e9
    traffic = None
    tsrc = None
    tpath = os.path.join(ROOT, "profiles", "uam_env_pmc.json") if uam else a.traffic
    if not uam and tpath and N != 5:     # per-N env PMC files (config 4: env_step_pmc_n8.json)
        tpath = tpath.replace(".json", f"_n{N}.json")
    if tpath and os.path.exists(tpath):
        with open(tpath) as f:
            t = json.load(f)
        if t.get("envs") == a.envs and t.get("agents") == N and (
                bool(t.get("tdcpa")) if uam else (t.get("variant", "att") == ("wgru" if tr.gru else "att") and
                                                  t.get("radar") == ("obstacles" if tr.gru else a.radar) and
                                                  t.get("maps", 1) == a.maps and
                                                  bool(t.get("tail", False)) == tr.fused_tail)):
            traffic = t.get("hbm_bytes_per_launch")
            tsrc = os.path.relpath(tpath, ROOT)
    if uam:
        upd_fl = uam_update_flops(a.batch)
        workload = (f"tdCPA_forV2_changeskin_UAM: {N} aircraft x {a.envs} envs/GPU, drifting cloud + go-around "
                    f"aircraft, tdCPA outputs live, float64 shared actor / single critic, B={a.batch}, "
                    f"1 gradient iteration per update")
    elif tr.gru:      # algorithmic GEMM FLOPs of the plan's launches (2 M N K per product)
        from multi_agent_aac_amd.fused import GemmLaunch
        from multi_agent_aac_amd.gru import WsProj
        upd_fl = sum(op.flops for op in tr.model._plan(a.batch).ops() if isinstance(op, (GemmLaunch, WsProj)))
        workload = f"randomOD_gru_radar: {N} agents x {a.envs} envs/GPU, GRU actor, B={a.batch} MADDPG update, " \
                   f"randomOD_Wgru_radar env (obstacle radar, per-agent WGRU ss_reward, max_spd 10)"
    else:
        upd_fl = update_flops(N, D0, a.batch)
        workload = f"one_model_att: {N} agents x {a.envs} envs/GPU, B={a.batch} MADDPG update, {a.radar} radar"
    if not uam and a.maps > 1:
        workload += f", {a.maps}-map stack (map drawn per env episode)"
    peak = FP64_PEAK_TFLOPS if uam else FP32_PEAK_TFLOPS
    out = {
        "metric": METRIC_UAM if uam else (METRIC_GRU if tr.gru else METRIC), "value": value,
        "unit": "agent-env-steps/s", "n_gpus": ws, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64 env + f64 learner" if uam else "f64 env state / f32 obs+learner",
        "data": "synthetic",
        "config": {"workload": workload, "envs_per_gpu": a.envs, "envs_total": E_total, "agents": N,
                   "batch": a.batch, "replay": a.memory, "radar": "runway+bound+clouds+aircraft" if uam else ("obstacles" if tr.gru else a.radar),
                   "parallelism": f"env-shard x{ws}" + (" + RCCL grad all-reduce" if ws > 1 else ""),
                   "maps": 1 if uam else a.maps, "tdcpa": uam,
                   "update_graph": (not a.no_graph) and (ws == 1 or uam or tr.gru or tr.model.fused),
                   "step_graph": (f"{group} steps per graph replay" if pairs else graphed),
                   "auto_reset": ("packed launch on a side stream beside the update" if _trainer.UAM_OVERLAP_RESET
                                  else "packed launch before the update") if uam else (
                                  "in the env step launch" if tr.fused_tail else "separate launch"),
                   "graph_segments": "one per update" if (ws == 1 or parallel.capturable(pg)) else
                   "cut at each gradient all-reduce"},
        "updates_per_s": upd_per_s, "grad_iters_per_s": upd_per_s * (1 if (tr.gru or uam) else N),
        "env_roofline": {"kernel": "uam_step_kernel (fused UAM env step)" if uam else (
                             "step_kernel (env step + replay push + auto-reset, aac_env_step_tail)" if tr.fused_tail
                             else "step_kernel (fused env step)"),
                         "push_bytes_per_agent_step": push_bpa,
                         "bound": "hbm", "achieved": achieved,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": tsrc, "bytes_per_agent_step": bpa, "agents_per_launch": a.envs * N,
                         "avg_launch_ms": env_ms,
                         "exact_band_list": None if band is None else {"most_per_launch": band[0], "capacity": band[1]}},
        "update_roofline": {"bound": "mfma", "unit": "TFLOP/s", "flop_per_update": upd_fl,
                            "achieved": upd_fl * upd_per_s / 1e12, "peak": peak,
                            "frac": upd_fl * upd_per_s / 1e12 / peak, "note": "whole-step rate bound"},
    }
    if not uam and not tr.gru:
        # the env kernel's second roofline: fp64 arithmetic (SURVEY.md section 8(d) FLOP count), with
        # the fp64 VALU instruction counts of a PMC pass at this size when one is committed
        fl = env_fp64_flop_per_agent_step(N)
        ach = fl * a.envs * N / (env_ms * 1e-3) / 1e12
        f64 = {"bound": "fp64", "flop_per_agent_step": fl, "achieved": ach, "peak": FP64_PEAK_TFLOPS,
               "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS}
        ppath = os.path.join(ROOT, "profiles", "env_fp64_pmc.json")
        if os.path.exists(ppath):
            with open(ppath) as f:
                pm = json.load(f)
            k = pm.get("step_kernel")
            if k and pm.get("envs") == a.envs and pm.get("agents") == N and pm.get("radar") == a.radar:
                # measured fp64 VALU work (every lane counted: an upper bound) at this config
                fpl = k["fp64_flop_per_launch"]
                f64["pmc"] = {"fp64_insts_per_launch": k["fp64_insts_per_launch"], "fp64_flop_per_launch": fpl,
                              "fp64_flop_per_agent_step": fpl / (a.envs * N),
                              "achieved": fpl / (env_ms * 1e-3) / 1e12,
                              "frac": fpl / (env_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                              "valu_insts_per_launch": k.get("SQ_INSTS_VALU"),
                              "int64_insts_per_launch": k.get("SQ_INSTS_VALU_INT64")}
                f64["pmc_source"] = os.path.relpath(ppath, ROOT)
        out["env_roofline"]["fp64"] = f64
    if not uam and (tr.gru or tr.model.fused):
        rf = gemm_roofline(tr.model, a.batch)
        rf["traffic"] = None
        if a.gemm_traffic and os.path.exists(a.gemm_traffic):
            with open(a.gemm_traffic) as f:
                t = json.load(f)
            if t.get("envs") == a.envs and t.get("agents") == N and t.get("batch") == a.batch and \
                    t.get("model", "att") == a.model:
                rf["traffic"] = t.get("hbm_bytes_per_launch")
                rf["traffic_source"] = os.path.relpath(a.gemm_traffic, ROOT)
                rf["traffic_over_algorithmic"] = rf["traffic"] / rf["algorithmic_bytes_per_launch"]
        out["roofline"] = rf
        if not tr.gru:
            out["attn_roofline"] = attn_roofline(tr.model, a.batch,
                                                 traffic_file=os.path.join(ROOT, "profiles", "r05_attn_pmc.json"))
    else:
        out["roofline"] = out["env_roofline"]
    if rank == 0 and ws == 1 and a.env_micro:
        out["env_microbench"] = uam_env_microbench(1 << 16, N) if uam else env_microbench(
            a.env_micro, N, a.radar, variant="wgru" if a.model == "gru" else "att")
    if rank == 0 and ws == 1 and not uam and not tr.gru and a.seg_overhead:
        out["world_schedule"] = world_schedule_overhead(a.agents, a.batch)
        out["segmented_overhead_us"] = out["world_schedule"].get("segmented_overhead_us")
    if rank == 0 and cpu is not None:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
