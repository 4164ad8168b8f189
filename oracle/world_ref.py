"""World / spawn pools / A* / OD restatement (oracle side; TEST INFRASTRUCTURE ONLY).

Follows, as text:
  * ATT/grid:148-180        cell squares ``Point(ix*10, iy*10).buffer(5, cap_style=3)`` for the
                            cells whose centre lies inside ``bound``; occupied after
                            ``ndimage.binary_fill_holes``
  * ATT/env:103-133         ``world_map_2D`` (x-major, [i][j]) rebuilt from cell centroids
  * ATT/env:136-197         quadrant pools ``target_area1..4`` (note: centres with
                            y == y_segment fall through to pool 4 -- kept)
  * ATT/env:251-347         random OD, ``jps_find_path`` and turning-point refinement
  * ATT/jps_straight.py:17-72  the 4-connected A* actually used
"""
import math

import numpy as np

from .consts import BOUND, GRID_LEN, PB


def cell_centre(i, j, bound=BOUND, grid_len=GRID_LEN):
    """Centre of grid cell (i, j): (ceil(b0/g)+i)*g, (ceil(b2/g)+j)*g  (ATT/env:334-335)."""
    return ((i + math.ceil(bound[0] / grid_len)) * grid_len,
            (j + math.ceil(bound[2] / grid_len)) * grid_len)


def target_pools(occ, bound=BOUND, grid_len=GRID_LEN):
    """The four ``target_pool`` lists of free-cell centres (ATT/env:152-197), x-major order."""
    w, h = occ.shape
    x_seg = (bound[1] - bound[0]) / 2 + bound[0]
    y_seg = (bound[3] - bound[2]) / 2 + bound[2]
    pools = [[], [], [], []]
    for i in range(w):
        for j in range(h):
            if occ[i, j]:
                continue
            cx, cy = cell_centre(i, j, bound, grid_len)
            cx, cy = float(cx), float(cy)
            if cx in (bound[0], bound[1]) or cy in (bound[2], bound[3]):
                continue  # centroid intersects a boundary line (ATT/env:155-157)
            if cx < x_seg and cy < y_seg:
                pools[0].append((cx, cy))
            elif cx > x_seg and cy < y_seg:
                pools[1].append((cx, cy))
            elif cx > x_seg and cy > y_seg:
                pools[2].append((cx, cy))
            else:
                pools[3].append((cx, cy))
    return pools


class _Node:
    __slots__ = ("parent", "position", "g", "h", "f")

    def __init__(self, parent=None, position=None):
        self.parent = parent
        self.position = position
        self.g = 0
        self.h = 0
        self.f = 0

    def __eq__(self, other):
        return self.position == other.position


def jps_find_path(start, end, grid):
    """Restatement of ATT/jps_straight.py:17-72 (list-based A*, first-min-f, no re-open)."""
    open_list, closed_list = [], []
    start_node = _Node(None, start)
    end_node = _Node(None, end)
    open_list.append(start_node)
    while open_list:
        current_node = open_list[0]
        current_index = 0
        for index, item in enumerate(open_list):
            if item.f < current_node.f:
                current_node = item
                current_index = index
        open_list.pop(current_index)
        closed_list.append(current_node)
        if current_node == end_node:
            path = []
            cur = current_node
            while cur is not None:
                path.append(cur.position)
                cur = cur.parent
            return path[::-1]
        children = []
        for d in [(0, -1), (0, 1), (-1, 0), (1, 0)]:
            np_ = (current_node.position[0] + d[0], current_node.position[1] + d[1])
            if np_[0] > len(grid) - 1 or np_[0] < 0 or np_[1] > len(grid[len(grid) - 1]) - 1 or np_[1] < 0:
                continue
            if grid[np_[0]][np_[1]] != 0:
                continue
            children.append(_Node(current_node, np_))
        for child in children:
            if child in closed_list:
                continue
            child.g = current_node.g + 1
            child.h = abs(child.position[0] - end_node.position[0]) + abs(child.position[1] - end_node.position[1])
            child.f = child.g + child.h
            if child in open_list:
                continue
            open_list.append(child)
    return None


def refine_path(out_path):
    """Turning points of an A* path (ATT/env:321-331)."""
    refined = [out_path[0]]
    cur_heading = math.atan2(out_path[1][1] - out_path[0][1], out_path[1][0] - out_path[0][0])
    for k in range(2, len(out_path)):
        nxt = math.atan2(out_path[k][1] - out_path[k - 1][1], out_path[k][0] - out_path[k - 1][0])
        if cur_heading != nxt:
            refined.append(out_path[k - 1])
            cur_heading = nxt
    refined.append(out_path[-1])
    return refined


def od_waypoints(occ, start_xy, end_xy, bound=BOUND, grid_len=GRID_LEN):
    """Goal / waypoint list for one agent (ATT/env:308-340).

    Returns a list of [x, y] (python numbers); the first refined point is dropped when it
    equals the start position, exactly as the list comprehension at ATT/env:334-338.
    """
    ox = math.ceil(bound[0] / grid_len)
    oy = math.ceil(bound[2] / grid_len)
    s = (int(start_xy[0] / grid_len) - ox, int(start_xy[1] / grid_len) - oy)
    e = (int(end_xy[0] / grid_len) - ox, int(end_xy[1] / grid_len) - oy)
    grid = occ.astype(int).tolist()
    path = jps_find_path(s, e, grid)
    if path is None:
        return None
    refined = refine_path(path)
    ini = np.array(start_xy)
    return [[(p[0] + ox) * grid_len, (p[1] + oy) * grid_len] for p in refined
            if not np.array_equal(np.array([(p[0] + ox) * grid_len, (p[1] + oy) * grid_len]), ini)]


def start_separated(candidate, previous):
    """``all(norm(cand - p) > 2*pB for p in previous)``  (ATT/env:267)."""
    return all(np.linalg.norm(np.array(candidate) - p) > PB * 2 for p in previous)
