"""numpy fp64 restatement of MPE ``simple_spread`` as vendored by MADDPG_SS_baseV3 (TEST
INFRASTRUCTURE ONLY).  ``SS/`` = MADDPG_SS_baseV3.

Follows, as text:
  World constants          SS/env/multiagent/core.py:82-98   dim_p 2, dim_c 2 (scenario), dt 0.1,
                                                             damping 0.25, contact_force 1e2,
                                                             contact_margin 1e-3, mass 1, no max_speed
  MultiAgentEnv.step       SS/env/multiagent/environment.py:80-103  set actions, world.step, then
                                                             obs / reward / done per agent; shared
                                                             reward only if world.collaborative (False)
  _set_action              SS/env/multiagent/environment.py:150-200  (vendored edit) u = action[0:2],
                                                             u *= sensitivity 5; silent agents
  World.step               SS/env/multiagent/core.py:116-169  action force (no u_noise), pairwise
                                                             collision force for a < b over entities
                                                             (landmarks do not collide), integrate
  get_collision_force      SS/env/multiagent/core.py:172-195  penetration = logaddexp(0, -(d - dmin)/k) k
  simple_spread            SS/env/multiagent/scenarios/simple_spread.py:6-100  3 agents (size 0.15),
                                                             3 landmarks; reward = -sum_l min_a |a - l|
                                                             - 1 per agent a colliding with this agent
                                                             (the agent itself included, so always
                                                             at least -1); obs = [vel, pos, l - pos,
                                                             others' pos - pos, others' comm (zeros)]
The env never reports done (done_callback None).  Arithmetic mirrors numpy's element order and
dtypes (float32 action force, float64 state).
"""
import numpy as np

DT, DAMPING, CONTACT_FORCE, CONTACT_MARGIN, SENSITIVITY, SIZE = 0.1, 0.25, 1e2, 1e-3, 5.0, 0.15


def _norm(v):
    return np.sqrt(np.sum(np.square(v)))


def step(pos, vel, lmk, act):
    """One env step.  pos, vel (N, 2) f64 (updated copies returned), lmk (L, 2), act (N, 2)."""
    N = pos.shape[0]
    pos, vel = pos.copy(), vel.copy()
    # _set_action scales the policy's float32 row in place (u *= 5 keeps float32); the first
    # collision term promotes the force to float64 (f_a + p_force[a])
    force = []
    for i in range(N):
        u = np.array(act[i], dtype=np.float32)
        u *= SENSITIVITY
        force.append(u)
    for a in range(N):                                # apply_environment_force (agents only collide)
        for b in range(a + 1, N):
            delta = pos[a] - pos[b]
            dist = np.sqrt(np.sum(np.square(delta)))
            dist_min = SIZE + SIZE
            k = CONTACT_MARGIN
            pen = np.logaddexp(0, -(dist - dist_min) / k) * k
            f = CONTACT_FORCE * delta / dist * pen
            force[a] = f + force[a]
            force[b] = -f + force[b]
    for i in range(N):                                # integrate_state
        vel[i] = vel[i] * (1 - DAMPING)
        vel[i] += (force[i] / 1.0) * DT
        pos[i] += vel[i] * DT
    return pos, vel


def observe(pos, vel, lmk):
    N = pos.shape[0]
    out = []
    for i in range(N):
        parts = [vel[i], pos[i]] + [lmk[j] - pos[i] for j in range(lmk.shape[0])]
        parts += [pos[j] - pos[i] for j in range(N) if j != i]
        parts += [np.zeros(2) for j in range(N) if j != i]
        out.append(np.concatenate(parts))
    return np.stack(out)


def reward(pos, lmk):
    N = pos.shape[0]
    rew = np.zeros(N)
    for i in range(N):
        r = 0
        for l in lmk:
            dists = [np.sqrt(np.sum(np.square(pos[a] - l))) for a in range(N)]
            r = r - min(dists)
        for a in range(N):
            if _norm(pos[a] - pos[i]) < SIZE + SIZE:
                r = r - 1
        rew[i] = r
    return rew


def reset(rng, N=3, L=3):
    """reset_world (simple_spread.py:32-44): agents first, then landmarks, uniform(-1, 1)."""
    pos = np.stack([rng.uniform(-1, +1, 2) for _ in range(N)])
    lmk = np.stack([rng.uniform(-1, +1, 2) for _ in range(L)])
    return pos, np.zeros((N, 2)), lmk
