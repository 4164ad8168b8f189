"""CPU tests of the UAM oracle (oracle/uam_ref.py): its GEOS closed forms
against exact rational arithmetic on the float vertices, the radar formulation against an exact
clip, the reference's known values, the episode sampler's rules, and the native episode-bank
builder's rules (host code, no GPU)."""
import math
import random
from fractions import Fraction

import numpy as np
import pytest

from oracle import geos
from oracle import uam_ref as U


def test_closed_forms_vs_exact():
    """gons_meet (touching counts / strict) and gon_rect_overlap agree with the exact
    separating-axis test on the GEOS float vertices away from a 1e-9 band of the threshold."""
    rng = np.random.default_rng(0)
    n = 0
    for _ in range(40):
        c = rng.uniform(14, 26, 2)
        for R, strict in ((1.0, False), (3.0, True), (1.0, True)):
            ang = rng.uniform(0, 2 * math.pi)
            rr = (0.5 + R) * rng.uniform(0.97, 1.03)
            q = c + rr * np.array([math.cos(ang), math.sin(ang)])
            m = max(abs((q - c) @ np.array(nv)) for nv in U.NORMALS) - (0.5 + R) * U.APO
            if abs(m) < 1e-9:
                continue
            assert U.gons_meet(c, 0.5, q, R, strict) == U.gons_meet_exact(c, 0.5, q, R, strict)
            n += 1
        p = np.array([rng.uniform(17, 23), rng.uniform(9, 31)])
        assert U.gon_rect_overlap(p, 0.5, U.RUNWAY) == U.gon_rect_overlap_exact(p, 0.5, U.RUNWAY)
    assert n > 100


def test_touching_is_no_conflict():
    """polygons_single_cloud_conflict (UAM/util:291-297): a circle touching the runway edge is not
    a conflict; overlapping by 1e-6 is."""
    assert not U.gon_rect_overlap((17.5, 20.0), 0.5, U.RUNWAY)
    assert U.gon_rect_overlap((17.500001, 20.0), 0.5, U.RUNWAY)
    assert not U.gon_rect_overlap((17.4, 20.0), 0.5, U.RUNWAY)


def test_ray_gon_boundary_vs_exact():
    """The radar's nearest boundary point of a 64-gon: entry from outside, exit from inside
    (LineString.intersection(polygon.boundary), UAM/env:1429-1486), against an exact clip."""
    rng = np.random.default_rng(1)
    hits = 0
    for _ in range(150):
        p = rng.uniform(10, 30, 2)
        r = float(rng.choice([0.5, 1.0, 3.0]))
        c = p + rng.uniform(-6, 6, 2)
        ang = rng.uniform(0, 2 * math.pi)
        e = (c[0] + 5 * math.cos(ang), c[1] + 5 * math.sin(ang))
        d = U._seg_gon(tuple(c), e, p, r)
        poly = geos.circle_vertices(p[0], p[1], r)
        t_in = geos.segment_convex_entry_exact(tuple(c), e, poly)
        if t_in is None:
            assert d is None
            continue
        L = Fraction(5)   # |e - c| up to rounding
        if t_in > 0:
            assert d is not None and abs(d - float(t_in) * geos.point_dist(e[0], e[1], c[0], c[1])) < 1e-9
            hits += 1
        else:   # c inside: the exit point, if the segment leaves the polygon
            t_out = geos.segment_convex_entry_exact(e, tuple(c), poly)
            if t_out is not None and t_out > 0:
                exit_d = (1 - float(t_out)) * geos.point_dist(e[0], e[1], c[0], c[1])
                assert d is not None and abs(d - exit_d) < 1e-9
                hits += 1
        del L
    assert hits > 10


def test_reference_helpers():
    """calculate_bearing (UAM/util:321-334) and calculate_next_position (UAM/util:300-318)."""
    assert U.calculate_bearing(0, 0, 1, 0) == 360
    assert U.calculate_bearing(0, 0, 0, -1) == 90
    assert U.calculate_bearing(0, 0, -1, 0) == 180
    assert U.calculate_bearing(0, 0, 0, 1) == 270
    np.testing.assert_allclose(U.calculate_next_position(np.array([8.0, 30.0]), np.array([10.0, 10.0]), 0.4, 0.5),
                               np.array([8.0, 30.0]) + 0.2 * np.array([2.0, -20.0]) / math.hypot(2, 20))
    assert np.array_equal(U.calculate_next_position(np.array([9.5, 10.5]), np.array([10.0, 10.0]), 0.4, 0.5),
                          np.array([9.5, 10.5]))


def test_end_regions_known_answer():
    """generate_random_end_pos's region subtraction (UAM/util:188-237) for cloud_a (8, 30): the
    regions left of the runway, worked out by hand."""
    regs = U.end_regions(0, 16.0)
    assert all(r[1] <= 18 for r in regs)
    area = sum((r[1] - r[0]) * (r[3] - r[2]) for r in regs)
    # x in [5, 18] x y in [5, 35] minus the cloud zone [3,13]x[25,35] and the go-around zone
    # [15,25]x[15,25]; the subtraction emits pieces left of the zone full-height, so pieces overlap
    assert area > 0 and min(r[0] for r in regs) == 5 and max(r[3] for r in regs) == 35


def test_sample_episode_rules():
    py, npr = random.Random(3), np.random.RandomState(3)
    for _ in range(20):
        s, g, c0, c1 = U.sample_episode(16, py, npr)
        assert c0 in (0, 1) and c1 in (0, 1, 2, 3)
        dd = np.linalg.norm(s[:, None] - s[None], axis=-1) + np.eye(16) * 9
        assert dd.min() > 1.5
        for a in range(16):
            assert any(r[0] <= g[a, 0] <= r[1] and r[2] <= g[a, 1] <= r[3] for r in U.end_regions(c0, s[a, 0]))


def test_oracle_frozen_after_goal():
    """An aircraft that reached its goal stops moving (UAM/env:4775-4790) and keeps +50."""
    env = U.UAMEnv(3)
    st = np.array([[16.0, 16.0], [24.0, 24.0], [16.0, 24.0]])
    go = np.array([[16.2, 16.0], [30.0, 30.0], [10.0, 30.0]])
    env.reset(st, go, 0, 0)
    _, r, d, cg, bbc, mk, over = env.full_step(np.zeros((3, 2)))
    assert mk[0] & 8 and mk[0] & 16 and r[0] == 50.0 and cg[0]
    p = env.all_agents[0].pos.copy()
    _, r, *_ = env.full_step(np.ones((3, 2)))
    assert np.array_equal(env.all_agents[0].pos, p) and r[0] == 50.0


def test_native_bank_rules(native_lib):
    from multi_agent_aac_amd import uam
    from multi_agent_aac_amd import uam
    N = 16
    bk = uam.build_bank(256, N, seed=9)
    assert set(np.unique(bk.clouds[:, 0])) <= {0, 1} and set(np.unique(bk.clouds[:, 1])) <= {0, 1, 2, 3}
    for k in range(bk.n):
        s, g = bk.start[k], bk.goal[k]
        inz = ((s[:, 0] >= 15) & (s[:, 0] <= 17) | (s[:, 0] >= 23) & (s[:, 0] <= 25)) & (s[:, 1] >= 15) & (s[:, 1] <= 25)
        assert inz.all()
        dd = np.linalg.norm(s[:, None] - s[None], axis=-1) + np.eye(N) * 9
        assert dd.min() > 1.5
        for a in range(N):
            regs = U.end_regions(int(bk.clouds[k, 0]), s[a, 0])
            assert any(r[0] <= g[a, 0] <= r[1] and r[2] <= g[a, 1] <= r[3] for r in regs)


