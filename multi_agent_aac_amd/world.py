"""Static world: synthetic occupancy maps, spawn pools and the OD bank.

The reference builds its 23 x 13 occupancy grid from ``lakeSide.shp`` (ATT/grid:108-185), which
is not in the repository, so the map is synthetic: seeded rectangular blobs over the same
[455, 680] x [255, 385] crop with 10 m cells until ~20 % are occupied, then
``ndimage.binary_fill_holes`` exactly as ATT/grid:164.  Maps are x-major ``occ[i, j]`` with
cell (i, j) centred at ((46 + i) * 10, (26 + j) * 10) -- ATT/env:334-335.

The OD bank (random start/goal + A* waypoints, ATT/env:251-347) is built natively
(``aac_od_bank_build`` in libaac_env.so) and installed on the device for auto-reset.
"""
import ctypes
import math

import numpy as np
from scipy import ndimage

from . import _native

BOUND = (455.0, 680.0, 255.0, 385.0)   # ATT/params:32-36
CELL = 10.0                            # ATT/grid:138
GRID_W, GRID_H = 23, 13


def grid_shape(bound=BOUND, cell=CELL):
    """Cells whose centre lies inside ``bound`` (ATT/grid:172)."""
    w = int(math.floor(bound[1] / cell) - math.ceil(bound[0] / cell)) + 1
    h = int(math.floor(bound[3] / cell) - math.ceil(bound[2] / cell)) + 1
    return w, h


def _connected_free(occ):
    free = occ == 0
    lab, n = ndimage.label(free)
    return n == 1


def synthetic_map(seed=2026, density=0.20, shape=(GRID_W, GRID_H), max_tries=1000):
    """Seeded synthetic occupancy map (see module docstring).  Deterministic for a seed.

    Accepted maps keep all free cells 4-connected (so every OD pair has an A* path) and keep
    a free cell in every border column/row (so ``world_map_2D`` spans the full crop, as the
    reference's centroid-based rebuild at ATT/env:117-131 assumes).
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    w, h = shape
    for _ in range(max_tries):
        occ = np.zeros((w, h), dtype=np.uint8)
        while occ.mean() < density:
            bw, bh = (int(v) for v in rng.integers(1, 4, size=2))
            i = int(rng.integers(0, w - bw + 1))
            j = int(rng.integers(0, h - bh + 1))
            occ[i:i + bw, j:j + bh] = 1
        occ = ndimage.binary_fill_holes(occ).astype(np.uint8)
        if not _connected_free(occ):
            continue
        if occ[0, :].all() or occ[-1, :].all() or occ[:, 0].all() or occ[:, -1].all():
            continue
        pools = target_pools(occ)
        if min(len(p) for p in pools) < 4:
            continue
        return occ
    raise RuntimeError("could not generate a valid map")


def map_stack(seeds, density=0.20):
    """Stack of maps for multi-map configs (config 5: seeds 2026..2033)."""
    return np.stack([synthetic_map(s, density) for s in seeds])


def target_pools(occ, bound=BOUND, cell=CELL):
    """Free-cell centres per quadrant pool (ATT/env:152-197); y == y_segment goes to pool 4."""
    w, h = occ.shape
    ox, oy = math.ceil(bound[0] / cell), math.ceil(bound[2] / cell)
    xs = (bound[1] - bound[0]) / 2 + bound[0]
    ys = (bound[3] - bound[2]) / 2 + bound[2]
    pools = [[], [], [], []]
    for i in range(w):
        for j in range(h):
            if occ[i, j]:
                continue
            cx, cy = (i + ox) * cell, (j + oy) * cell
            if cx in (bound[0], bound[1]) or cy in (bound[2], bound[3]):
                continue
            q = 0 if (cx < xs and cy < ys) else 1 if (cx > xs and cy < ys) else 2 if (cx > xs and cy > ys) else 3
            pools[q].append((cx, cy))
    return pools


def astar(occ, start, end, max_len=4096):
    """A* path (list of (i, j)) via the native restatement of ATT/jps_straight.py."""
    occ = np.ascontiguousarray(occ, dtype=np.uint8)
    out = np.zeros((max_len, 2), dtype=np.int32)
    n = _native.lib().aac_astar(occ.ctypes.data, occ.shape[0], occ.shape[1], int(start[0]), int(start[1]),
                                int(end[0]), int(end[1]), out.ctypes.data, max_len)
    if n < 0:
        raise RuntimeError("aac_astar: invalid arguments")
    return [tuple(int(v) for v in out[k]) for k in range(n)] if n else None


class ODBank:
    """``n_pairs`` independent agent ODs drawn with the reference rule; waypoints padded to W."""

    def __init__(self, occ, n_pairs=65536, seed=2026, max_wp=32, bound=BOUND, cell=CELL):
        occ = np.ascontiguousarray(occ, dtype=np.uint8)
        self.start = np.zeros((n_pairs, 2), dtype=np.float64)
        self.wps = np.zeros((n_pairs, max_wp, 2), dtype=np.float64)
        self.cnt = np.zeros((n_pairs,), dtype=np.int32)
        b = np.asarray(bound, dtype=np.float64)
        rc = _native.lib().aac_od_bank_build(occ.ctypes.data, occ.shape[0], occ.shape[1], b.ctypes.data,
                                             ctypes.c_double(cell), n_pairs, ctypes.c_uint64(seed), max_wp,
                                             self.start.ctypes.data, self.wps.ctypes.data, self.cnt.ctypes.data)
        if rc < 0:
            raise RuntimeError(f"aac_od_bank_build failed ({rc})")
        if rc > max_wp:
            raise RuntimeError(f"OD bank needs {rc} waypoints > max_wp={max_wp}")
        self.max_seen = rc
        self.n_pairs, self.max_wp, self.seed = n_pairs, max_wp, seed

    def sample_env_od(self, E, N, rng, pb=2.5):
        """Host-side draw of E x N ODs with the start-separation rule (ATT/env:258-268)."""
        start = np.zeros((E, N, 2))
        wps = np.zeros((E, N, self.max_wp, 2))
        cnt = np.zeros((E, N), dtype=np.int32)
        for e in range(E):
            chosen = []
            for a in range(N):
                while True:
                    k = int(rng.integers(0, self.n_pairs))
                    s = self.start[k]
                    if all(np.linalg.norm(s - self.start[c]) > pb * 2 for c in chosen):
                        break
                chosen.append(k)
                start[e, a] = s
                wps[e, a] = self.wps[k]
                cnt[e, a] = self.cnt[k]
        return start, wps, cnt


class MapBanks:
    """One ``ODBank`` per map of a stack (the multipleMap variant draws the map per episode,
    multipleMap/ma_main:464-465, then the OD from that map, ATT/env:251-347), concatenated
    map-major for ``aac_env_set_od_banks``."""

    def __init__(self, occ_stack, n_pairs=65536, seed=2026, max_wp=32, bound=BOUND, cell=CELL):
        occ_stack = np.asarray(occ_stack, dtype=np.uint8)
        assert occ_stack.ndim == 3
        self.banks = [ODBank(o, n_pairs=n_pairs, seed=seed + 7919 * m, max_wp=max_wp, bound=bound, cell=cell)
                      for m, o in enumerate(occ_stack)]
        self.n_maps, self.max_wp = len(self.banks), max_wp
        self.start = np.ascontiguousarray(np.concatenate([b.start for b in self.banks]))
        self.wps = np.ascontiguousarray(np.concatenate([b.wps for b in self.banks]))
        self.cnt = np.ascontiguousarray(np.concatenate([b.cnt for b in self.banks]))
        self.counts = np.array([b.n_pairs for b in self.banks], dtype=np.int32)
        self.offsets = np.concatenate([[0], np.cumsum(self.counts)]).astype(np.int64)
