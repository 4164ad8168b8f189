"""Shared helpers for the parity tests (OD drawing via the oracle restatement, padding)."""
import numpy as np

from oracle import world_ref

W_DEFAULT = 32


def draw_env_od(occ, N, rng, pools=None):
    """One env's OD by the reference rule (ATT/env:251-347), via the oracle restatement."""
    pools = pools or world_ref.target_pools(occ)
    starts, goals = [], []
    for _ in range(N):
        while True:
            qs = int(rng.integers(0, 4))
            qt = int(rng.choice([q for q in range(4) if q != qs]))
            s = pools[qs][int(rng.integers(0, len(pools[qs])))]
            if world_ref.start_separated(s, [np.array(p) for p in starts]):
                break
        t = pools[qt][int(rng.integers(0, len(pools[qt])))]
        starts.append(s)
        goals.append(world_ref.od_waypoints(occ, s, t))
    return starts, goals


def pack_od(od_list, W=W_DEFAULT):
    """[(starts, goals)] per env -> start (E,N,2), wps (E,N,W,2), cnt (E,N)."""
    E, N = len(od_list), len(od_list[0][0])
    st = np.zeros((E, N, 2))
    wps = np.zeros((E, N, W, 2))
    cnt = np.zeros((E, N), dtype=np.int32)
    for e, (s, g) in enumerate(od_list):
        for i in range(N):
            st[e, i] = s[i]
            wps[e, i, :len(g[i])] = g[i]
            wps[e, i, len(g[i]):] = g[i][-1]
            cnt[e, i] = len(g[i])
    return st, wps, cnt


def random_od(occ, E, N, seed, W=W_DEFAULT):
    rng = np.random.default_rng(seed)
    pools = world_ref.target_pools(occ)
    return pack_od([draw_env_od(occ, N, rng, pools) for _ in range(E)], W)


def mix64(x):
    """splitmix64 finaliser used by the GPU auto-reset draw (csrc/aac_env.hip ``mix64``)."""
    M = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & M
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & M
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & M
    return x ^ (x >> 31)


MAP_DRAW_KEY = 0x6d61705f64726177


def map_draw(seed, e, episode, n_maps):
    """The auto-reset's per-episode map of env e with per-map banks (csrc/aac_env.hip reset_kernel)."""
    return mix64(mix64(mix64(seed ^ MAP_DRAW_KEY ^ e) ^ episode)) % n_maps


def bank_draw(bank_start, n_bank, seed, e, episode, N, pb=2.5, off=0):
    """Python restatement of the auto-reset draw (starts pairwise > 2 pB apart) from the bank
    entries off .. off + n_bank - 1."""
    idx = []
    for a in range(N):
        k = 0
        for att in range(4096):
            key = mix64(mix64(mix64(seed ^ e) ^ episode) ^ (a * 65536 + att))
            k = off + key % n_bank
            s = bank_start[k]
            ok = True
            for b in idx:
                o = bank_start[b]
                d = np.sqrt(np.fma(s[1] - o[1], s[1] - o[1], (s[0] - o[0]) * (s[0] - o[0]))) if hasattr(np, "fma") \
                    else np.linalg.norm(s - o)
                if not d > pb * 2:
                    ok = False
                    break
            if ok:
                break
        idx.append(k)
    return idx


_M64 = np.uint64((1 << 64) - 1)


def mix64_np(x):
    """``mix64`` over a uint64 array (numpy wraps uint64 arithmetic modulo 2^64)."""
    x = np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def bank_draw_batch(bank_start, n_bank, seed, envs, episodes, N, pb=2.5, off=0):
    """``bank_draw`` for many envs at once (vectorised over envs): returns the drawn bank indices
    (len(envs), N).  Separation distances within 1e-9 of the 2 pB threshold are re-decided by the
    scalar rule (np.linalg.norm of a 2-vector, the kernel's fma form)."""
    envs = np.asarray(envs, dtype=np.uint64)
    eps = np.asarray(episodes, dtype=np.uint64)
    M = len(envs)
    idx = np.zeros((M, N), dtype=np.int64)
    if M == 0:
        return idx
    h0 = mix64_np(mix64_np(np.uint64(seed) ^ envs) ^ eps)
    chosen = np.zeros((M, N, 2))
    for a in range(N):
        pick = np.full(M, -1, dtype=np.int64)
        last = np.zeros(M, dtype=np.int64)
        for att0 in range(0, 4096, 64):
            todo = np.nonzero(pick < 0)[0]
            if len(todo) == 0:
                break
            att = np.arange(att0, att0 + 64, dtype=np.uint64)
            key = mix64_np(h0[todo, None] ^ (np.uint64(a * 65536) + att)[None, :])
            k = off + (key % np.uint64(n_bank)).astype(np.int64)         # (T, 64)
            s = bank_start[k]                                               # (T, 64, 2)
            ok = np.ones(k.shape, dtype=bool)
            for b in range(a):
                o = chosen[todo, b][:, None, :]
                d = np.sqrt((s[..., 0] - o[..., 0]) ** 2 + (s[..., 1] - o[..., 1]) ** 2)
                near = np.abs(d - 2 * pb) < 1e-9
                ok &= d > 2 * pb
                for ti, j in zip(*np.nonzero(near)):       # the exact rule at the threshold
                    ok[ti, j] = all(np.linalg.norm(s[ti, j] - chosen[todo[ti], bb]) > 2 * pb for bb in range(a))
            first = np.where(ok.any(1), ok.argmax(1), -1)
            hit = first >= 0
            pick[todo[hit]] = k[hit, first[hit]]
            last[todo] = k[:, 63]
        pick = np.where(pick < 0, last, pick)
        idx[:, a] = pick
        chosen[:, a] = bank_start[pick]
    return idx


def uam_oracle_steps(pre, acts, N):
    """Worker for the config-5 parity test (spawned process, numpy only): one oracle/uam_ref.py
    step per env of ``pre`` (a device state dict sliced to the checked envs) from that exact
    pre-step state.  Returns [(obs, reward, done, check_goal, bbc, mask, over, post_state, tdcpa)]."""
    from oracle import uam_ref as U
    out = []
    for e in range(len(acts)):
        o = U.env_from_state(pre, e, N)
        res = o.full_step(acts[e])
        out.append(tuple(res) + (U.state_of(o), o.tdcpa_out))
    return out


def wgru_targets(wp, wp_rm, wp_cnt):
    """First remaining waypoint of every agent of the WGRU variant (wp_rm: removal bit mask)."""
    W = wp.shape[2]
    k = np.arange(W)
    valid = (k < np.asarray(wp_cnt)[..., None]) & (((np.asarray(wp_rm, np.int64)[..., None] >> k) & 1) == 0)
    first = np.argmax(valid, -1)
    return np.take_along_axis(wp, first[..., None, None].repeat(2, -1), 2)[:, :, 0]


def steer(pos, vel, target, rng, noise=0.3, gain=0.15, damp=0.4):
    """Actions in [-1, 1] that fly toward ``target`` with noise (exercises waypoint / goal events)."""
    a = gain * (target - pos) - damp * vel + noise * rng.standard_normal(pos.shape)
    return np.clip(a, -1, 1).astype(np.float32)
