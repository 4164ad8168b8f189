"""Vectorised NumPy restatement of the ``one_model_att`` env step over E envs (TEST INFRASTRUCTURE and
CPU BASELINE ONLY: BASELINE.md's "mode 2", timed by bench.py's cpu_baseline leg).

The same algorithm and formulas as oracle/aac_oracle.c / oracle/env_ref.py (which follow ATT/env
line by line: kinematics ATT/env:2639-2713, radar ATT/env:1051-1170 + OM/env:1049-1148, observation
ATT/env:1285-1469, ss_reward ATT/env:2105-2603, termination ATT/main:448-462), evaluated as array
operations over (env, agent, ray, neighbour / cell / edge) instead of per-agent Python loops.  NumPy
has no fused multiply-add, so ``np.linalg.norm`` (whose OpenBLAS ddot tail is an FMA) is
``sqrt(x*x + y*y)`` here: values may differ from the C oracle in the last bits, never in a
decision away from a tie (tests/test_oracle_cpu.py::test_numpy_env_matches_c_oracle).

``variant="wgru"``: the randomOD_Wgru_radar env of config 4 (oracle/wgru_env_ref.py, WGRU/env:824-2131,
WGRU/ma_main:653-661) -- obstacle radar, 6-wide own rows, per-agent reward against the next waypoint and
the reference path, the goal list as removed-waypoint bits in ``wp_cur``.

Threshold bands (oracle/geos.py BAND, BAND_T): the elements whose closed form lies within the band of
its threshold -- a goal or building separating-axis margin, a radar clip interval, a slab tie -- are
decided again by the scalar geos functions (their exact fallbacks), as in the C oracle and the kernel.
"""
import math

import numpy as np

from . import geos
from .consts import ACC_MAX, BOUND, DT, GRID_LEN, EPISODE_LENGTH, MATH_PI, PB, RADAR_DIST, VMAX

N_RAYS = 18
_RAD = np.array([20 * r * (MATH_PI / 180.0) for r in range(N_RAYS)])
RAY_C, RAY_S = np.cos(_RAD), np.sin(_RAD)
_INC = abs(0.0 - 2.0 * MATH_PI) / int(abs(0.0 - 2.0 * MATH_PI) / (MATH_PI / 2.0 / 16) + 0.5)
CIRC_C = np.cos(0.0 + (-1.0 * np.arange(64)) * _INC)
CIRC_S = np.sin(0.0 + (-1.0 * np.arange(64)) * _INC)
NRM_C = np.cos((np.arange(64) + 0.5) * MATH_PI / 32.0)
NRM_S = np.sin((np.arange(64) + 0.5) * MATH_PI / 32.0)
APOTHEM = math.cos(MATH_PI / 64.0)
QUANTUM = MATH_PI / 2.0 / 16


def _norm(x, y):
    return np.sqrt(x * x + y * y)


class NumpyEnv:
    """E x N envs; state arrays as the GPU handle / C oracle (SoA, float64)."""

    def __init__(self, E, N, occ, W=32, radar_mode=2, compat=True, episode_length=EPISODE_LENGTH, bound=BOUND,
                 variant="att"):
        self.E, self.N, self.K, self.W = E, N, N - 1, W
        self.wgru = variant == "wgru"
        if self.wgru:
            from .wgru_env_ref import EPISODE_LENGTH as WL, VMAX as WV
            radar_mode, self.vmax = 1, float(WV)
            episode_length = WL if episode_length == EPISODE_LENGTH else episode_length
        else:
            self.vmax = float(VMAX)
        self.D0 = 6 if self.wgru else 6 + 4 * self.K
        self.mode, self.compat, self.T = radar_mode, compat, episode_length
        self.b = np.array(bound, dtype=np.float64)
        occ = np.asarray(occ, dtype=np.uint8)
        self.occ = occ
        gx0, gy0 = math.ceil(self.b[0] / GRID_LEN) * GRID_LEN, math.ceil(self.b[2] / GRID_LEN) * GRID_LEN
        self.gx0, self.gy0 = gx0, gy0
        ii, jj = np.nonzero(occ)
        self.cells = np.stack([gx0 + 10.0 * ii, gy0 + 10.0 * jj], 1)          # occupied cell centres
        z = lambda *s: np.zeros(s)   # noqa: E731
        self.pos, self.vel, self.pre_pos, self.pre_vel, self.goal, self.start = (z(E, N, 2) for _ in range(6))
        self.wp = z(E, N, W, 2)
        self.wp_cur = np.zeros((E, N), np.int64)
        self.wp_cnt = np.zeros((E, N), np.int64)
        self.reach = np.zeros((E, N), bool)
        self.wall = np.zeros((E, N), np.int64)
        self.step_count = np.zeros(E, np.int64)
        self.others = np.array([[j for j in range(N) if j != i] for i in range(N)])      # (N, K)

    # ------------------------------------------------------------------ reset
    def reset(self, start, wps, cnt, env_mask=None):
        m = np.ones(self.E, bool) if env_mask is None else np.asarray(env_mask, bool)
        self.pos[m] = start[m]
        self.pre_pos[m] = start[m]
        self.start[m] = start[m]
        self.vel[m] = 0.0
        self.pre_vel[m] = 0.0
        self.wp[m] = wps[m]
        self.wp_cnt[m] = cnt[m]
        self.wp_cur[m] = 0
        idx = (cnt[m] - 1)[..., None, None]
        self.goal[m] = np.take_along_axis(wps[m], np.broadcast_to(idx, idx.shape[:2] + (1, 2)), 2)[:, :, 0]
        self.reach[m] = False
        self.wall[m] = 0
        self.step_count[m] = 0
        return self.observe()

    # ------------------------------------------------------------------ observation
    def _radar(self, sl):
        p = self.pos[sl]                                    # (e, N, 2)
        px, py = p[..., 0][..., None], p[..., 1][..., None]   # (e, N, 1)
        ex, ey = px + RADAR_DIST * RAY_C, py + RADAR_DIST * RAY_S           # (e, N, R)
        ln = _norm(ex - px, ey - py)
        ddx, ddy = ex - px, ey - py
        dd = ln.copy()
        if self.mode != 1:                                  # drones: Cyrus-Beck against the 64-gons
            q = p[:, self.others]                           # (e, N, K, 2)
            vx = q[..., 0][..., None] + PB * CIRC_C          # (e, N, K, 64)
            vy = q[..., 1][..., None] + PB * CIRC_S
            wx, wy = np.roll(vx, -1, -1), np.roll(vy, -1, -1)
            exx, eyy = (wx - vx)[:, :, None], (wy - vy)[:, :, None]       # (e, N, 1, K, 64)
            cx, cy = px[..., None, None], py[..., None, None]
            a = exx * (cy - vy[:, :, None]) - eyy * (cx - vx[:, :, None])
            bb = exx * ddy[..., None, None] - eyy * ddx[..., None, None]  # (e, N, R, K, 64)
            with np.errstate(divide="ignore", invalid="ignore"):
                t = -a / bb
            tlo = np.maximum(np.where(bb < 0, t, 0.0).max(-1), 0.0)
            thi = np.minimum(np.where(bb > 0, t, 1.0).min(-1), 1.0)
            hit = ~((bb == 0) & (a > 0)).any(-1) & (tlo <= thi)
            for idx in zip(*np.nonzero(~((bb == 0) & (a > 0)).any(-1) & (np.abs(tlo - thi) <= geos.BAND_T)
                                       & (tlo < 1.0 - geos.BAND_T))):
                e, i, r, k = idx                           # threshold band: the scalar clip + exact test
                c = (float(px[e, i, 0]), float(py[e, i, 0]))
                qq = q[e, i, k]
                t = geos.ray_polygon_entry(c[0], c[1], float(ex[e, i, r]), float(ey[e, i, r]),
                                           geos.circle_vertices(float(qq[0]), float(qq[1]), PB))
                hit[idx] = t is not None
                tlo[idx] = t if t is not None else tlo[idx]
            ix, iy = px[..., None] + tlo * ddx[..., None], py[..., None] + tlo * ddy[..., None]
            d = np.where(hit, _norm(ix - px[..., None], iy - py[..., None]), np.inf)
            dmin = d.min(-1)
            dd = np.where(np.isfinite(dmin), dmin, ln)
        dob = ln.copy()
        if self.mode != 0:                                  # obstacles: slab test per occupied cell
            C = self.cells
            x0, x1 = C[:, 0] - 5.0, C[:, 0] + 5.0
            y0, y1 = C[:, 1] - 5.0, C[:, 1] + 5.0
            cx, cy = px[..., None], py[..., None]
            dx_, dy_ = ddx[..., None], ddy[..., None]
            with np.errstate(divide="ignore", invalid="ignore"):
                ta, tb = (x0 - cx) / dx_, (x1 - cx) / dx_
                tx0, tx1 = np.where(dx_ == 0, -np.inf, np.minimum(ta, tb)), np.where(dx_ == 0, np.inf, np.maximum(ta, tb))
                ta, tb = (y0 - cy) / dy_, (y1 - cy) / dy_
                ty0, ty1 = np.where(dy_ == 0, -np.inf, np.minimum(ta, tb)), np.where(dy_ == 0, np.inf, np.maximum(ta, tb))
            okx = (dx_ != 0) | ((cx >= x0) & (cx <= x1))
            oky = (dy_ != 0) | ((cy >= y0) & (cy <= y1))
            tin, tout = np.maximum(tx0, ty0), np.minimum(tx1, ty1)
            ok = okx & oky & ~((tin > tout) | (tout < 0.0) | (tin > 1.0))
            t = np.where(tin >= 0.0, tin, tout)
            ok &= t <= 1.0
            on_edge = ((dx_ == 0) & ((cx == x0) | (cx == x1)) & (cy >= y0) & (cy <= y1)) | \
                      ((dy_ == 0) & ((cy == y0) | (cy == y1)) & (cx >= x0) & (cx <= x1))
            d = np.where(on_edge, 0.0, np.where(ok, _norm((cx + t * dx_) - cx, (cy + t * dy_) - cy), np.inf))
            band = ~on_edge & (np.abs(tin - tout) <= geos.BAND_T) & (tin < 1.0 - geos.BAND_T)
            for idx in zip(*np.nonzero(band)):          # threshold band: the scalar slab + exact test
                e, i, r, k = idx
                v = geos.ray_square_crossing(float(px[e, i, 0]), float(py[e, i, 0]), float(ex[e, i, r]),
                                             float(ey[e, i, r]), float(x0[k]), float(x1[k]), float(y0[k]), float(y1[k]))
                d[idx] = np.inf if v is None else v
            dob = np.minimum(dob, d.min(-1)) if len(C) else dob
            b = self.b
            for lx in (b[0], b[1]):
                col = (px == lx) & (ex == lx)
                with np.errstate(divide="ignore", invalid="ignore"):
                    t = (lx - px) / (ex - px)
                    dl = np.where(col, 0.0, _norm(lx - px, (py + t * (ey - py)) - py))
                hitl = col | ((px - lx) * (ex - lx) <= 0.0)
                dob = np.where(hitl & (dl < dob), dl, dob)
            for ly in (b[2], b[3]):
                col = (py == ly) & (ey == ly)
                with np.errstate(divide="ignore", invalid="ignore"):
                    t = (ly - py) / (ey - py)
                    dl = np.where(col, 0.0, _norm((px + t * (ex - px)) - px, ly - py))
                hitl = col | ((py - ly) * (ey - ly) <= 0.0)
                dob = np.where(hitl & (dl < dob), dl, dob)
        if self.mode == 0:
            return dd
        if self.mode == 1:
            return dob
        return np.where(dd < dob, dd, dob)

    def observe(self, chunk=256):
        E, N, K, b = self.E, self.N, self.K, self.b
        XS, YS = 2.0 / (b[1] - b[0]), 2.0 / (b[3] - b[2])
        p, v, g = self.pos, self.vel, self.goal
        npx, npy = -1 + (p[..., 0] - b[0]) * XS, -1 + (p[..., 1] - b[2]) * YS
        ngx = 2 * ((g[..., 0] - b[0]) / (b[1] - b[0])) - 1
        ngy = 2 * ((g[..., 1] - b[2]) / (b[3] - b[2])) - 1
        VM = self.vmax
        own = np.zeros((E, N, self.D0))
        own[..., 0], own[..., 1] = npx, npy
        if self.wgru:                                   # scale_vel (WGRU/env:971)
            own[..., 2], own[..., 3] = XS * v[..., 0], YS * v[..., 1]
        else:
            own[..., 2], own[..., 3] = v[..., 0] / VM, v[..., 1] / VM
        own[..., 4], own[..., 5] = ngx - npx, ngy - npy
        q, w = p[:, self.others], v[:, self.others]                 # (E, N, K, 2)
        dx, dy = q[..., 0] - p[..., None, 0], q[..., 1] - p[..., None, 1]
        if self.compat:
            g0, g1 = w[..., 1] - q[..., 0], PB - q[..., 1]
        else:
            gq = g[:, self.others]
            g0, g1 = gq[..., 0] - q[..., 0], gq[..., 1] - q[..., 1]
        if not self.wgru:
            if self.compat:
                own[..., 6::4], own[..., 7::4] = -1 + (dx - b[0]) * XS, -1 + (dy - b[2]) * YS
            else:
                own[..., 6::4], own[..., 7::4] = XS * dx, YS * dy
            own[..., 8::4], own[..., 9::4] = w[..., 0] / VM, w[..., 1] / VM
        dxm, dxM, dym, dyM = b[0] - b[1], b[1] - b[0], b[2] - b[3], b[3] - b[2]
        nei = np.zeros((E, N, K, 6))
        nei[..., 0], nei[..., 1] = 2 * ((dx - dxm) / (dxM - dxm)) - 1, 2 * ((dy - dym) / (dyM - dym)) - 1
        nei[..., 2], nei[..., 3] = 2 * ((g0 - dxm) / (dxM - dxm)) - 1, 2 * ((g1 - dym) / (dyM - dym)) - 1
        nei[..., 4], nei[..., 5] = w[..., 0] / VM, w[..., 1] / VM
        radar = np.concatenate([self._radar(slice(s, s + chunk)) for s in range(0, E, chunk)])
        self.radar64 = radar
        return own.astype(np.float32), radar.astype(np.float32), nei.astype(np.float32)

    # ------------------------------------------------------------------ step
    def _bound_crash(self):
        p0, p1, r, b = self.pre_pos, self.pos, PB, self.b
        x0, y0, x1, y1 = p0[..., 0], p0[..., 1], p1[..., 0], p1[..., 1]
        same = (x0 == x1) & (y0 == y1)
        dx, dy = x1 - x0, y1 - y0
        ln = np.sqrt(dx * dx + dy * dy)
        with np.errstate(divide="ignore", invalid="ignore"):
            ux, uy = 1 * r * dx / ln, 1 * r * dy / ln
        xs = [x1 - uy, x1 + uy, x0 + uy, x0 - uy]
        ys = [y1 + ux, y1 - ux, y0 - ux, y0 + ux]
        k = np.arange(1, 32)
        for (cx, cy, a) in ((x1, y1, np.arctan2(dy, dx)), (x0, y0, np.arctan2(y0 - y1, x0 - x1))):
            st, en = a + MATH_PI / 2.0, a - MATH_PI / 2.0
            inc = np.abs(st - en) / np.floor(np.abs(st - en) / QUANTUM + 0.5)
            ang = st[..., None] + (-1.0 * k) * inc[..., None]
            xs.append(cx[..., None] + r * np.cos(ang))
            ys.append(cy[..., None] + r * np.sin(ang))
        X = np.concatenate([x[..., None] if x.ndim == 2 else x for x in xs], -1)
        Y = np.concatenate([y[..., None] if y.ndim == 2 else y for y in ys], -1)
        Xc, Yc = x0[..., None] + r * CIRC_C, y0[..., None] + r * CIRC_S
        mnx = np.where(same, Xc.min(-1), X.min(-1))
        mxx = np.where(same, Xc.max(-1), X.max(-1))
        mny = np.where(same, Yc.min(-1), Y.min(-1))
        mxy = np.where(same, Yc.max(-1), Y.max(-1))
        return ((mnx <= b[0]) & (b[0] <= mxx)) | ((mnx <= b[1]) & (b[1] <= mxx)) | \
               ((mny <= b[2]) & (b[2] <= mxy)) | ((mny <= b[3]) & (b[3] <= mxy))

    def _goal(self, g, dxg, dyg):
        """goal 64-gon predicate (ATT/env:2266-2269); the threshold band by the scalar exact fallback."""
        m = (dxg[..., None] * NRM_C + dyg[..., None] * NRM_S).max(-1)
        thr = (PB + 1.0) * APOTHEM
        goal = m <= thr
        for e, a in zip(*np.nonzero(np.abs(m - thr) <= geos.BAND)):
            goal[e, a] = geos.goal_reached(float(self.pos[e, a, 0]), float(self.pos[e, a, 1]),
                                           float(g[e, a, 0]), float(g[e, a, 1]))
        return goal

    def _building(self):
        p = self.pos
        ci = np.floor((p[..., 0] - self.gx0) / 10.0 + 0.5).astype(np.int64)
        cj = np.floor((p[..., 1] - self.gy0) / 10.0 + 0.5).astype(np.int64)
        gw, gh = self.occ.shape
        hit = np.zeros(p.shape[:2], bool)
        lim = 5.0 * (np.abs(NRM_C[:32]) + np.abs(NRM_S[:32])) + PB * APOTHEM
        for di in (-1, 0, 1):
            for dj in (-1, 0, 1):
                ii, jj = ci + di, cj + dj
                inb = (ii >= 0) & (jj >= 0) & (ii < gw) & (jj < gh)
                occ = np.zeros_like(inb)
                occ[inb] = self.occ[ii[inb], jj[inb]] != 0
                dx, dy = (self.gx0 + 10.0 * ii) - p[..., 0], (self.gy0 + 10.0 * jj) - p[..., 1]
                near = (np.abs(dx) <= 5.0 + PB) & (np.abs(dy) <= 5.0 + PB)
                proj = np.abs(dx[..., None] * NRM_C[:32] + dy[..., None] * NRM_S[:32])
                h = inb & occ & near & (proj <= lim).all(-1)
                lim0 = 5.0 + PB
                band = inb & occ & ((np.abs(np.abs(dx) - lim0) <= geos.BAND) | (np.abs(np.abs(dy) - lim0) <= geos.BAND)
                                    | (np.abs(proj - lim) <= geos.BAND).any(-1))
                for e, a in zip(*np.nonzero(band)):     # threshold band: the scalar test + exact fallback
                    h[e, a] = geos.building_hit_cell(float(p[e, a, 0]), float(p[e, a, 1]),
                                                     float(self.gx0 + 10.0 * ii[e, a]), float(self.gy0 + 10.0 * jj[e, a]))
                hit |= h
        return hit

    def step(self, act):
        """Kinematics + observation + ss_reward + termination; returns (own, radar, nei, reward,
        done, mask, env_done, bbc) like the GPU step."""
        a = np.asarray(act, dtype=np.float32).astype(np.float64) * ACC_MAX
        self.pre_pos[:] = self.pos
        self.pre_vel[:] = self.vel
        cvx, cvy = self.vel[..., 0] + a[..., 0] * DT, self.vel[..., 1] + a[..., 1] * DT
        nh = np.arctan2(cvy, cvx)
        VM = self.vmax
        fast = _norm(cvx, cvy) >= VM
        self.vel[..., 0] = np.where(fast, VM * np.cos(nh), cvx)
        self.vel[..., 1] = np.where(fast, VM * np.sin(nh), cvy)
        self.pos = self.pos + self.vel * DT
        own, radar, nei = self.observe()
        if self.wgru:
            return (own, radar, nei) + self._wgru_reward()
        p, N = self.pos, self.N
        q = p[:, self.others]
        dist = _norm(p[..., None, 0] - q[..., 0], p[..., None, 1] - q[..., 1])     # (E, N, K)
        shortest = dist.min(-1)
        nearest = self.others[np.arange(N)[None, :], dist.argmin(-1)]
        coll = dist <= PB * 2
        ncoll = coll.sum(-1)
        last = np.where(coll.any(-1), self.others[np.arange(N)[None, :], (coll.shape[-1] - 1) - np.argmax(coll[..., ::-1], -1)], -1)
        c_drone, m_drone = 1 + (2.5 / (10 - 2.5)), (0 - 1) / (10 - 2.5)
        band = (dist >= 2.5) & (dist <= 10)
        pen = np.zeros(shortest.shape)
        for k in range(self.K):                       # sequential, as the reference loop
            pen = pen + np.where(band[..., k], 1 * (m_drone * shortest + c_drone), 0)
        building = self._building()
        self.wall += building
        g = self.goal
        dxg, dyg = g[..., 0] - p[..., 0], g[..., 1] - p[..., 1]
        goal = self._goal(g, dxg, dyg)
        w0 = np.take_along_axis(self.wp, self.wp_cur[..., None, None].repeat(2, -1), 2)[:, :, 0]
        wpf = _norm(p[..., 0] - w0[..., 0], p[..., 1] - w0[..., 1]) < 5
        before = _norm(self.pre_pos[..., 0] - g[..., 0], self.pre_pos[..., 1] - g[..., 1])
        after = _norm(p[..., 0] - g[..., 0], p[..., 1] - g[..., 1])
        dtg = (1 * (before - after)) / 5
        bnd = self._bound_crash()
        mask = bnd.astype(np.uint8) | (ncoll > 0) << 1 | goal << 2 | building << 3 | wpf << 4
        r = np.where(bnd, ((0.0 - 20) - 0.0) - 0,
                     np.where(ncoll > 0, ((0.0 - 20) - 0.0) - pen, np.where(goal, (0.0 + 20) + 0.0, dtg - pen)))
        done = bnd | (ncoll > 0)
        cg = ~bnd & ~(ncoll > 0) & goal
        normal = ~bnd & ~(ncoll > 0) & ~goal
        self.reach |= cg
        adv = normal & wpf & (self.wp_cnt - self.wp_cur > 1)
        self.wp_cur = np.where(adv, self.wp_cur + 1, self.wp_cur)
        mask = mask | (cg.astype(np.uint8) << 5)
        team = r[:, 0].copy()
        for i in range(1, N):                         # numpy pairwise sum is sequential below 8
            team = team + r[:, i]
        if N >= 8:
            team = np.sum(r, axis=1)
        reward = np.repeat(team[:, None], N, 1).astype(np.float32)
        bbc = np.zeros((self.E, 4), np.uint8)
        bbc[:, 0] = bnd.any(1)
        bbc[:, 2] = (~bnd & (ncoll > 0)).any(1)
        bbc[:, 3] = (~bnd & (ncoll > 0) & (last == nearest)).any(1)
        self.step_count += 1
        env_done = (self.T < self.step_count) | done.any(1) | cg.all(1) | self.reach.all(1)
        return own, radar, nei, reward, done.astype(np.uint8), mask.astype(np.uint8), env_done.astype(np.uint8), bbc

    # ------------------------------------------------------------------ WGRU ss_reward
    def _wgru_reward(self):
        """WGRU/env:1666-2039 over all agents (the loop forms of oracle/wgru_env_ref.py as array ops)."""
        E, N, W = self.E, self.N, self.W
        p, pp, v = self.pos, self.pre_pos, self.vel
        px, py = p[..., 0], p[..., 1]
        q = p[:, self.others]
        dist = _norm(px[..., None] - q[..., 0], py[..., None] - q[..., 1])
        ncoll = (dist <= PB * 2).sum(-1)
        building = self._building()
        self.wall += building
        g = self.goal
        goal = self._goal(g, g[..., 0] - px, g[..., 1] - py)
        # next waypoint (:1815-1832): the first strict running minimum below 5 stops the scan
        k = np.arange(W)
        rm = self.wp_cur
        valid = (k < self.wp_cnt[..., None]) & (((rm[..., None] >> k) & 1) == 0)
        d = np.where(valid, _norm(px[..., None] - self.wp[..., 0], py[..., None] - self.wp[..., 1]), np.inf)
        pm = np.concatenate([np.full((E, N, 1), np.inf), np.minimum.accumulate(d, -1)[..., :-1]], -1)
        trig = valid & (d < pm) & (d < 5)
        flag = trig.any(-1)
        kt = np.argmax(trig, -1)
        nrem = valid.sum(-1)
        pop = flag & (nrem > 1)
        rm = np.where(pop, rm | (np.int64(1) << kt), rm)
        nrem = nrem - pop
        valid2 = valid & ~(pop[..., None] & (k == kt[..., None]))
        d2 = np.where(valid2, _norm(self.wp[..., 0] - px[..., None], self.wp[..., 1] - py[..., None]), np.inf)
        nxt_k = np.where(pop, np.argmin(d2, -1), np.where(flag, kt, np.argmin(d, -1)))
        nxt = np.take_along_axis(self.wp, nxt_k[..., None, None].repeat(2, -1), 2)[:, :, 0]
        self.wp_cur = rm
        last = (W - 1) - np.argmax(valid2[..., ::-1], -1)               # goal[-1] after the pop
        self.goal = np.take_along_axis(self.wp, last[..., None, None].repeat(2, -1), 2)[:, :, 0].copy()
        dtg = 1 * (_norm(pp[..., 0] - nxt[..., 0], pp[..., 1] - nxt[..., 1]) - _norm(px - nxt[..., 0], py - nxt[..., 1]))
        # cross-track distance to the path start, wp[0..cnt) (WGRU/env:2621-2632, GEOS DistanceOp)
        P = np.concatenate([self.start[:, :, None], self.wp], 2)           # (E, N, W + 1, 2)
        ax, ay, bx, by = P[..., :-1, 0], P[..., :-1, 1], P[..., 1:, 0], P[..., 1:, 1]
        X, Y = px[..., None], py[..., None]
        with np.errstate(divide="ignore", invalid="ignore"):
            len2 = (bx - ax) * (bx - ax) + (by - ay) * (by - ay)
            r = ((X - ax) * (bx - ax) + (Y - ay) * (by - ay)) / len2
            sv = ((ay - Y) * (bx - ax) - (ax - X) * (by - ay)) / len2
            dA, dB = _norm(X - ax, Y - ay), _norm(X - bx, Y - by)
            dseg = np.where((ax == bx) & (ay == by), dA, np.where(r <= 0.0, dA, np.where(r >= 1.0, dB,
                                                                                       np.abs(sv) * np.sqrt(len2))))
            f = np.where((X == ax) & (Y == ay), 0.0, np.where((X == bx) & (Y == by), 1.0, r))
        segv = k < self.wp_cnt[..., None]
        ks = np.argmin(np.where(segv, dseg, np.inf), -1)[..., None]
        pick = lambda a: np.take_along_axis(a, ks, -1)[..., 0]   # noqa: E731
        fs, Ax, Ay, Bx, By = pick(f), pick(ax), pick(ay), pick(bx), pick(by)
        inside = (fs > 0) & (fs < 1)
        d0, d1 = _norm(Ax - px, Ay - py), _norm(Bx - px, By - py)
        qx = np.where(inside, Ax + fs * (Bx - Ax), np.where(d0 < d1, Ax, Bx))
        qy = np.where(inside, Ay + fs * (By - Ay), np.where(d0 < d1, Ay, By))
        cross = _norm(px - qx, py - qy)
        dref = np.where(cross <= PB, 3 * (((0 - 1) / (PB - 0)) * cross + 1), -3 * 1)
        thr = 2 * PB
        ssp = 3 * ((thr - np.clip(_norm(v[..., 0], v[..., 1]), 0, thr)) * (1.0 / thr))
        rmin = self.radar64.min(-1)
        nbp = np.where((rmin >= PB) & (rmin <= 5), 3 * (((0 - 1) / (5 - PB)) * rmin + 2), 0.0)
        bnd = self._bound_crash()
        crash = (((((0.0 + dref) - 5) + dtg) - ssp) + 0.0) - nbp
        normal = (((((np.where(flag & (nrem > 1), 3.0, 0.0) + dref) + dtg) - ssp) + 0.0) - nbp) + 0.0
        r = np.where(bnd | (building != 0), crash, np.where(goal, (0.0 + 5) + 0.0, normal))
        done = bnd | (building != 0)
        cg = ~done & goal
        self.reach |= cg
        mask = (bnd.astype(np.uint8) | (ncoll > 0) << 1 | goal << 2 | (building != 0) << 3 | flag << 4
                | cg.astype(np.uint8) << 5)
        bbc = np.zeros((E, 4), np.uint8)
        bbc[:, 0] = bnd.any(1)
        bbc[:, 1] = (~bnd & (building != 0)).any(1)
        self.step_count += 1
        env_done = (self.T < self.step_count) | done.any(1) | self.reach.all(1)
        return (r.astype(np.float32), done.astype(np.uint8), mask.astype(np.uint8), env_done.astype(np.uint8), bbc)
