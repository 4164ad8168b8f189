"""Generate the committed golden vectors tests/golden/env_*.npz from the reference-shaped scalar
oracle (oracle/env_ref.py, which follows ATT/env line by line).  Inputs are the reference's own
fixed-OD fixtures (fixed_od.json, extracted from MA_ver1/fixedDrone_*.xlsx) or seeded random OD,
on the synthetic map (seed 2026); actions are either a deterministic go-to-waypoint controller
(drives agents into goal / waypoint / head-on collision events) or seeded U[-1, 1].

Run:  python tests/golden/make_golden.py   (deterministic; rewrites the .npz files)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import env_ref, world_ref  # noqa: E402

W = 32


def synthetic_map():
    from multi_agent_aac_amd import world
    return world.synthetic_map(2026)


def controller(env):
    a = []
    for i, ag in env.all_agents.items():
        d = np.array(ag.waypoints[0], dtype=float) - ag.pos
        n = np.linalg.norm(d)
        a.append(d / n if n > 0 else np.zeros(2))
    return np.array(a, dtype=np.float32)


def run(occ, N, od_list, mode, T, actions="controller", seed=0):
    E = len(od_list)
    envs = [env_ref.ScalarEnv(N, occ, radar_mode=mode) for _ in range(E)]
    st = np.zeros((E, N, 2)); wps = np.zeros((E, N, W, 2)); cnt = np.zeros((E, N), np.int32)
    for e, (s, g) in enumerate(od_list):
        for i in range(N):
            st[e, i] = s[i]; wps[e, i, :len(g[i])] = g[i]; wps[e, i, len(g[i]):] = g[i][-1]; cnt[e, i] = len(g[i])
    rec = {k: [] for k in ("act", "own", "radar", "nei", "reward", "mask", "done", "env_done", "bbc", "pos", "vel")}
    init = [env.reset(od_list[e][0], od_list[e][1]) for e, env in enumerate(envs)]
    rng = np.random.default_rng(seed)
    alive = np.ones(E, bool)
    for t in range(T):
        if actions == "controller":
            act = np.stack([controller(env) for env in envs])
        else:
            act = rng.uniform(-1, 1, size=(E, N, 2)).astype(np.float32)
        outs = [env.full_step(act[e]) for e, env in enumerate(envs)]
        rec["act"].append(act)
        rec["own"].append(np.stack([o[0][0] for o in outs]).astype(np.float32))
        rec["radar"].append(np.stack([o[0][1] for o in outs]).astype(np.float32))
        rec["nei"].append(np.stack([o[0][2] for o in outs]).astype(np.float32))
        rec["reward"].append(np.array([[float(x) for x in o[1]] for o in outs], dtype=np.float32))
        rec["done"].append(np.array([o[2] for o in outs], dtype=np.uint8))
        rec["bbc"].append(np.array([o[4] for o in outs], dtype=np.uint8))
        rec["mask"].append(np.array([o[5] for o in outs], dtype=np.uint8))
        rec["env_done"].append(np.array([o[6] for o in outs], dtype=np.uint8))
        rec["pos"].append(np.stack([[env.all_agents[i].pos for i in range(N)] for env in envs]))
        rec["vel"].append(np.stack([[env.all_agents[i].vel for i in range(N)] for env in envs]))
        alive &= ~rec["env_done"][-1].astype(bool)
        if not alive.any():
            break
    out = {k: np.stack(v) for k, v in rec.items()}
    out.update(occ=occ, start=st, wps=wps, cnt=cnt, radar_mode=np.int32(mode),
               own0=np.stack([i[0] for i in init]).astype(np.float32),
               radar0=np.stack([i[1] for i in init]).astype(np.float32),
               nei0=np.stack([i[2] for i in init]).astype(np.float32))
    return out


def main():
    occ = synthetic_map()
    fixed = json.load(open(os.path.join(HERE, "fixed_od.json")))
    scen = {}
    for name, key, mode in (("fixed3", "fixedDrone_3drones.xlsx", 0), ("fixed5", "fixedDrone_5_adj.xlsx", 2)):
        ag = fixed[key]["agents"]
        od = ([tuple(a["start"]) for a in ag], [a["goals"] for a in ag])
        scen[name] = run(occ, len(ag), [od], mode, T=60)
    rng = np.random.default_rng(2026)
    pools = world_ref.target_pools(occ)

    def rand_od(N):
        from tests.helpers import draw_env_od
        return draw_env_od(occ, N, rng, pools)

    scen["rand5_drones"] = run(occ, 5, [rand_od(5) for _ in range(4)], 0, T=30, actions="random", seed=1)
    scen["rand8_obstacles"] = run(occ, 8, [rand_od(8) for _ in range(3)], 1, T=30, actions="random", seed=2)
    scen["ctrl5_combined"] = run(occ, 5, [rand_od(5) for _ in range(4)], 2, T=60, actions="controller")
    # the remaining reference fixtures (appended: the scenarios above keep their random streams).
    # fixedDrone_2_drone / fixedDrone_3drones_2 are head-on pairs: the go-to-waypoint controller
    # flies them into each other (drone collision, bbc[2] / bbc[3])
    for name, key, mode, T in (("headon2", "fixedDrone_2_drone.xlsx", 2, 40),
                               ("headon2_long", "fixedDrone_3drones_2.xlsx", 0, 60),
                               ("fixed5_all", "fixedDrone.xlsx", 0, 60),
                               ("fixed3v2", "fixedDrone_3dronesV2.xlsx", 1, 60)):
        ag = fixed[key]["agents"]
        od = ([tuple(a["start"]) for a in ag], [a["goals"] for a in ag])
        scen[name] = run(occ, len(ag), [od], mode, T=T)
    for k, v in scen.items():
        np.savez_compressed(os.path.join(HERE, f"env_{k}.npz"), **v)
        m = np.bitwise_or.reduce(v["mask"].ravel())
        print(k, "steps", v["act"].shape[0], "mask bits seen", bin(int(m)), "env_done", int(v["env_done"].sum()))


if __name__ == "__main__":
    main()
