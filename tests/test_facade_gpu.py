"""The two boundaries on the GPU:

* the committed golden vectors (tests/golden/env_*.npz, produced by the reference-shaped scalar
  oracle from the reference's fixed-OD fixtures and seeded OD) replayed through the C ABI;
* the drop-in facades (``env_simulator`` / ``MADDPG`` / ``ReplayMemory``) driven by a loop shaped
  like ATT/main:225-460 against the scalar oracle (oracle/env_ref.py) on identical actions.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import env_ref

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ATOL = 1e-5


@pytest.mark.parametrize("name", ["fixed3", "fixed5", "rand5_drones", "rand8_obstacles", "ctrl5_combined",
                                  "headon2", "headon2_long", "fixed5_all", "fixed3v2"])
def test_goldens_through_abi(native_lib, name):
    from multi_agent_aac_amd.env import BatchedEnv
    g = np.load(os.path.join(GOLDEN, f"env_{name}.npz"))
    E, N = g["start"].shape[:2]
    env = BatchedEnv(E, N, g["occ"], radar_mode=int(g["radar_mode"]), max_wp=g["wps"].shape[2])
    env.reset(g["start"], g["wps"], g["cnt"])
    torch.cuda.synchronize()
    b = env.bufs
    for k in ("own", "radar", "nei"):
        np.testing.assert_allclose(getattr(b, k).cpu().numpy(), g[k + "0"], rtol=0, atol=ATOL, err_msg=k + "0")
    for t in range(g["act"].shape[0]):
        env.step(torch.from_numpy(g["act"][t]).cuda())
        torch.cuda.synchronize()
        for k in ("own", "radar", "nei", "reward"):
            np.testing.assert_allclose(getattr(b, k).cpu().numpy(), g[k][t], rtol=0, atol=ATOL,
                                       err_msg=f"{name} t{t} {k}")
        for k in ("mask", "done", "env_done", "bbc"):
            assert np.array_equal(getattr(b, k).cpu().numpy(), g[k][t]), (name, t, k)
        np.testing.assert_allclose(env.get_state()["pos"].cpu().numpy(), g["pos"][t], rtol=0, atol=1e-9)


def _norm_lists_close(a, b):
    """Compare two norm_state lists [[own_i], [radar_i], [[nei_ik (1, 6)]]] (ATT/env:1483-1491)."""
    for i in range(len(a[0])):
        np.testing.assert_allclose(np.asarray(a[0][i], np.float64), np.asarray(b[0][i], np.float64), atol=ATOL)
        np.testing.assert_allclose(np.asarray(a[1][i], np.float64), np.asarray(b[1][i], np.float64), atol=ATOL)
        for k in range(len(a[2][i])):
            np.testing.assert_allclose(np.asarray(a[2][i][k], np.float64).ravel(),
                                       np.asarray(b[2][i][k], np.float64).ravel(), atol=ATOL)


def test_facade_ma_main_loop(native_lib, occ):
    from multi_agent_aac_amd.env import env_simulator
    from multi_agent_aac_amd.maddpg import MADDPG

    fixed = json.load(open(os.path.join(GOLDEN, "fixed_od.json")))["fixedDrone_5_adj.xlsx"]["agents"]
    starts = [tuple(a["start"]) for a in fixed]
    goals = [a["goals"] for a in fixed]
    N = len(fixed)
    acc_max, max_spd = 8, 5                                             # ATT/main:136-150
    env = env_simulator(occ, radar_mode="drones", seed=1)
    env.create_world(N, 2, 0.95, 0.01, 1, 0.5, 0.15, 0.5, None, max_spd, [-acc_max, acc_max])
    with pytest.warns(UserWarning):
        model = MADDPG([16, 18, 6], [16, 18, 6], 2, 64, 10, N, None, 1e-3, 1e-3, 0.95, 0.01, True,
                       seed=0, memory_length=1000, batch_size=32)
    ref = env_ref.ScalarEnv(N, occ, radar_mode=0)
    cur_state, norm_cur = env.reset_world(N, [16, 18, 6], show=0, starts=starts, goals=goals)
    o = ref.reset(starts, goals)
    _norm_lists_close(norm_cur, [list(o[0]), list(o[1]), [[o[2][i, k][None] for k in range(N - 1)]
                                                          for i in range(N)]])
    p0 = model.fa.data.clone()
    losses = []
    episodes, step, total = 1, 0, 0
    for _ in range(90):
        action, _, _, _ = model.choose_action(norm_cur, total, episodes, step, 8000, 1.0, None, noisy=True)
        nxt, norm_nxt, *_ = env.step(action, step, acc_max, [16, 18, 6])
        rew, done, check_goal, _, _, _, bbc = env.ss_reward(step, [[] for _ in range(N)], None,
                                                            [[] for _ in range(N)], (None, None), True, None)
        (ro, rr, rn), rrew, rdone, rcg, rbbc, rmask, over = ref.full_step(np.asarray(action, np.float32))
        _norm_lists_close(norm_nxt, [list(ro), list(rr), [[rn[i, k][None] for k in range(N - 1)] for i in range(N)]])
        np.testing.assert_allclose(rew, [float(x) for x in rrew], atol=ATOL)
        assert done == [bool(x) for x in rdone] and check_goal == [bool(x) for x in rcg]
        assert bbc == [bool(x) for x in rbbc]
        for i in range(N):
            np.testing.assert_allclose(env.all_agents[i].pos, ref.all_agents[i].pos, rtol=0, atol=1e-9)
            assert len(env.all_agents[i].waypoints) == len(ref.all_agents[i].waypoints)
        # ATT/main:363-400: push the normalised transition, then update_myown
        model.memory.push(norm_cur, action, norm_nxt, np.array(rew), np.array(done, np.float32))
        c_loss, a_loss, _ = model.update_myown(episodes, total, 1, [])
        if c_loss is not None:
            losses.append(float(c_loss[0]))
        step += 1
        total += 1
        norm_cur = norm_nxt
        if over or step > 50:
            episodes += 1
            step = 0
            cur_state, norm_cur = env.reset_world(N, [16, 18, 6], show=0, starts=starts, goals=goals)
            ref.reset(starts, goals)
    assert len(model.memory) == 90
    assert losses and np.isfinite(losses).all()
    assert not torch.equal(p0, model.fa.data)
