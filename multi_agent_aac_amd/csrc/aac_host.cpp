// aac_host.cpp -- host-side world utilities of libaac_env.so: the A* of ATT/jps_straight.py and
// the OD bank (random OD + A* waypoints, ATT/env:251-347) that feeds GPU auto-reset.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#include "../../include/aac_env.h"

namespace {

struct Node {
    int x, y, g, f, parent;
};

// ATT/jps_straight.py:17-72: list-based open set, first strictly-smaller f wins, children in
// order (0,-1),(0,1),(-1,0),(1,0), children already open are skipped (no g re-relaxation).
int astar(const uint8_t *grid, int w, int h, int sx, int sy, int ex, int ey, std::vector<int> &path) {
    std::vector<Node> pool;
    std::vector<int> open;                  // indices into pool, in list order
    std::vector<uint8_t> closed(w * h, 0), in_open(w * h, 0);
    pool.push_back({sx, sy, 0, 0, -1});
    open.push_back(0);
    in_open[sx * h + sy] = 1;
    static const int dirs[4][2] = {{0, -1}, {0, 1}, {-1, 0}, {1, 0}};
    while (!open.empty()) {
        size_t ci = 0;
        for (size_t k = 1; k < open.size(); ++k)
            if (pool[open[k]].f < pool[open[ci]].f) ci = k;
        int cur = open[ci];
        open.erase(open.begin() + ci);
        Node cn = pool[cur];
        in_open[cn.x * h + cn.y] = 0;
        closed[cn.x * h + cn.y] = 1;
        if (cn.x == ex && cn.y == ey) {
            path.clear();
            for (int n = cur; n >= 0; n = pool[n].parent) {
                path.push_back(pool[n].x);
                path.push_back(pool[n].y);
            }
            // reverse pairs
            std::vector<int> rev(path.size());
            for (size_t k = 0; k < path.size() / 2; ++k) {
                rev[2 * k] = path[path.size() - 2 - 2 * k];
                rev[2 * k + 1] = path[path.size() - 1 - 2 * k];
            }
            path.swap(rev);
            return (int)(path.size() / 2);
        }
        for (auto &d : dirs) {
            int nx = cn.x + d[0], ny = cn.y + d[1];
            if (nx > w - 1 || nx < 0 || ny > h - 1 || ny < 0) continue;
            if (grid[nx * h + ny] != 0) continue;
            if (closed[nx * h + ny]) continue;
            if (in_open[nx * h + ny]) continue;
            int g = cn.g + 1;
            int hh = std::abs(nx - ex) + std::abs(ny - ey);
            pool.push_back({nx, ny, g, g + hh, cur});
            open.push_back((int)pool.size() - 1);
            in_open[nx * h + ny] = 1;
        }
    }
    return 0;
}

}  // namespace

extern "C" int aac_astar(const uint8_t *grid, int32_t w, int32_t h, int32_t sx, int32_t sy, int32_t ex, int32_t ey,
                         int32_t *path_xy, int32_t max_len) {
    if (!grid || w <= 0 || h <= 0) return AAC_E_INVALID;
    std::vector<int> p;
    int n = astar(grid, w, h, sx, sy, ex, ey, p);
    for (int k = 0; k < n && k < max_len; ++k) {
        path_xy[2 * k] = p[2 * k];
        path_xy[2 * k + 1] = p[2 * k + 1];
    }
    return n;
}

extern "C" int aac_od_bank_build(const uint8_t *occ, int32_t w, int32_t h, const double *bound, double cell,
                                 int32_t n_pairs, uint64_t seed, int32_t max_wp, double *start, double *wps,
                                 int32_t *cnt) {
    if (!occ || !bound || !start || !wps || !cnt || n_pairs <= 0 || max_wp < 1) return AAC_E_INVALID;
    const int ox = (int)std::ceil(bound[0] / cell), oy = (int)std::ceil(bound[2] / cell);
    const double xseg = (bound[1] - bound[0]) / 2 + bound[0], yseg = (bound[3] - bound[2]) / 2 + bound[2];
    std::vector<int> pools[4];   // cell index i*h + j, x-major order (ATT/env:152-197)
    for (int i = 0; i < w; ++i)
        for (int j = 0; j < h; ++j) {
            if (occ[i * h + j]) continue;
            double cx = (i + ox) * cell, cy = (j + oy) * cell;
            if (cx == bound[0] || cx == bound[1] || cy == bound[2] || cy == bound[3]) continue;
            int q;
            if (cx < xseg && cy < yseg) q = 0;
            else if (cx > xseg && cy < yseg) q = 1;
            else if (cx > xseg && cy > yseg) q = 2;
            else q = 3;
            pools[q].push_back(i * h + j);
        }
    for (auto &p : pools)
        if (p.empty()) return AAC_E_INVALID;
    std::mt19937_64 rng(seed);
    int max_seen = 0;
    std::vector<int> path;
    for (int32_t k = 0; k < n_pairs; ++k) {
        int qs = (int)(rng() % 4);
        int qt = (int)(rng() % 3);
        if (qt >= qs) ++qt;
        int s = pools[qs][rng() % pools[qs].size()];
        int t = pools[qt][rng() % pools[qt].size()];
        int sx = s / h, sy = s % h, tx = t / h, ty = t % h;
        int n = astar(occ, w, h, sx, sy, tx, ty, path);
        if (n < 2) return AAC_E_STATE;   // unreachable pair: the reference would crash (outPath None)
        // turning points (ATT/env:321-331), start point dropped (:334-338)
        std::vector<int> ref;
        ref.push_back(0);
        int hx = path[2] - path[0], hy = path[3] - path[1];
        for (int m = 2; m < n; ++m) {
            int nx = path[2 * m] - path[2 * m - 2], ny = path[2 * m + 1] - path[2 * m - 1];
            if (nx != hx || ny != hy) {
                ref.push_back(m - 1);
                hx = nx;
                hy = ny;
            }
        }
        ref.push_back(n - 1);
        start[2 * k] = (sx + ox) * cell;
        start[2 * k + 1] = (sy + oy) * cell;
        int c = 0;
        for (int m : ref) {
            double x = (path[2 * m] + ox) * cell, y = (path[2 * m + 1] + oy) * cell;
            if (x == start[2 * k] && y == start[2 * k + 1]) continue;
            if (c < max_wp) {
                wps[((size_t)k * max_wp + c) * 2] = x;
                wps[((size_t)k * max_wp + c) * 2 + 1] = y;
            }
            ++c;
        }
        for (int r = c; r < max_wp; ++r) {   // pad with the final goal
            wps[((size_t)k * max_wp + r) * 2] = wps[((size_t)k * max_wp + (c < max_wp ? c : max_wp) - 1) * 2];
            wps[((size_t)k * max_wp + r) * 2 + 1] = wps[((size_t)k * max_wp + (c < max_wp ? c : max_wp) - 1) * 2 + 1];
        }
        cnt[k] = c < max_wp ? c : max_wp;
        if (c > max_seen) max_seen = c;
    }
    return max_seen;
}
