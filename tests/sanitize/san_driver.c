/* san_driver.c -- AddressSanitizer / UndefinedBehaviorSanitizer run of the host-side C/C++ (SURVEY.md
 * section 5 "race detection / sanitizers"): the A* and OD-bank builder of libaac_env.so
 * (multi_agent_aac_amd/csrc/aac_host.cpp) and the C oracle (oracle/aac_oracle.c, included whole so its
 * internal helpers run too).  Built by `make -C oracle sanitize`, run by tests/test_sanitize_cpu.py.
 * No GPU code: HIP kernels cannot run under ASan on this pool.  Exit 0 = no finding. */
#include "../../oracle/aac_oracle.c"
#include "../../include/aac_env.h"

#include <stdio.h>

static uint64_t lcg = 0x9E3779B97F4A7C15ull;
static double urand(void) {
    lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
    return (double)(lcg >> 11) * (1.0 / 9007199254740992.0);
}

int main(void) {
    enum { GW = 23, GH = 13, P = 2048, W = 32 };
    const double bound[4] = {455.0, 680.0, 255.0, 385.0};
    static uint8_t occ[GW * GH];
    /* a few walls with gaps: every free cell stays reachable */
    for (int j = 2; j < 11; ++j) occ[6 * GH + j] = (j != 6);
    for (int j = 1; j < 9; ++j) occ[15 * GH + j] = 1;
    for (int i = 9; i < 13; ++i) occ[i * GH + 4] = 1;
    /* A* on every pair of a sample of cells, including occupied start / end cells */
    static int32_t path[2 * GW * GH];
    long total = 0;
    for (int k = 0; k < 4000; ++k) {
        int sx = (int)(urand() * GW), sy = (int)(urand() * GH), ex = (int)(urand() * GW), ey = (int)(urand() * GH);
        int n = aac_astar(occ, GW, GH, sx, sy, ex, ey, path, GW * GH);
        if (n < 0) { fprintf(stderr, "astar error %d\n", n); return 2; }
        total += n;
    }
    /* the OD bank: starts, waypoints (padded), counts */
    double *start = malloc(sizeof(double) * 2 * P), *wps = malloc(sizeof(double) * 2 * P * W);
    int32_t *cnt = malloc(sizeof(int32_t) * P);
    int mx = aac_od_bank_build(occ, GW, GH, bound, 10.0, P, 7, W, start, wps, cnt);
    if (mx < 1 || mx > W) { fprintf(stderr, "od bank %d\n", mx); return 3; }
    /* the C oracle: both variants, every radar mode, reset from bank entries, random steps */
    for (int variant = 0; variant < 2; ++variant)
        for (int mode = 0; mode < 3; ++mode) {
            const int E = 24, N = variant ? 8 : 5, K = N - 1, D0 = variant ? 6 : 6 + 4 * K;
            oc_cfg cfg = {E, N, W, variant ? 1 : mode, 1, variant ? 0 : 1, variant ? 150 : 50, GW, GH,
                          {bound[0], bound[1], bound[2], bound[3]}, occ, 1, variant, variant ? 10.0 : 5.0};
            double *pos = calloc(E * N * 2, 8), *vel = calloc(E * N * 2, 8), *ppos = calloc(E * N * 2, 8);
            double *pvel = calloc(E * N * 2, 8), *goal = calloc(E * N * 2, 8), *wp = calloc(E * N * W * 2, 8);
            double *st = calloc(E * N * 2, 8), *swp = calloc(E * N * W * 2, 8);
            int32_t *cur = calloc(E * N, 4), *wc = calloc(E * N, 4), *wall = calloc(E * N, 4), *stp = calloc(E, 4);
            int32_t *scnt = calloc(E * N, 4), *midx = calloc(E, 4);
            uint8_t *reach = calloc(E * N, 1);
            oc_state s = {pos, vel, ppos, pvel, goal, wp, cur, wc, reach, wall, stp, midx, calloc(E * N * 2, 8)};
            float *own = calloc(E * N * D0, 4), *radar = calloc(E * N * NRAY, 4), *nei = calloc(E * N * K * 6, 4);
            float *rew = calloc(E * N, 4), *act = calloc(E * N * 2, 4);
            uint8_t *done = calloc(E * N, 1), *mask = calloc(E * N, 1), *edone = calloc(E, 1), *bbc = calloc(E * 4, 1);
            double *tcpa = calloc(E * N * K, 8), *dcpa = calloc(E * N * K, 8);
            int32_t *cc = calloc(E * N, 4), *cp = calloc(E * N, 4);
            oc_out out = {own, radar, nei, rew, done, mask, edone, bbc, tcpa, dcpa, cc, cp};
            for (int e = 0; e < E; ++e)
                for (int i = 0; i < N; ++i) {
                    int b = (e * N + i) * 37 % P;
                    st[(e * N + i) * 2] = start[2 * b] + 0.37 * i;     /* separated starts */
                    st[(e * N + i) * 2 + 1] = start[2 * b + 1];
                    memcpy(&swp[(size_t)(e * N + i) * W * 2], &wps[(size_t)b * W * 2], sizeof(double) * W * 2);
                    scnt[e * N + i] = cnt[b];
                }
            oc_reset(&cfg, &s, NULL, st, swp, scnt, NULL, &out);
            for (int t = 0; t < 60; ++t) {
                for (int k = 0; k < E * N * 2; ++k) act[k] = (float)(2.0 * urand() - 1.0);
                oc_step(&cfg, &s, act, &out);
                oc_reset(&cfg, &s, edone, st, swp, scnt, NULL, &out);
            }
            free(pos); free(vel); free(ppos); free(pvel); free(goal); free(wp); free(st); free(swp); free(cur);
            free(wc); free(wall); free(stp); free(scnt); free(midx); free(reach); free(s.start); free(own);
            free(radar); free(nei); free(rew); free(act); free(done); free(mask); free(edone); free(bbc);
            free(tcpa); free(dcpa); free(cc); free(cp);
        }
    /* the exact threshold fallbacks: goals on the apothem, circles on cell edges, capsules on the bound */
    init_tables();
    int hits = 0;
    for (int k = 0; k < 64; ++k) {
        double a = (k + 0.5) * PI_GEOS / 32.0, r = 3.5 * cos(PI_GEOS / 64.0);
        hits += oc_goal_reached(600.0, 330.0, 600.0 + r * cos(a), 330.0 + r * sin(a));
        hits += oc_building_hit(527.5, 310.0 + 0.1 * k, 520.0, 310.0);
        hits += oc_bound_crash(457.5, 300.0 + k, 457.5, 300.0 + k, bound);
    }
    free(start); free(wps); free(cnt);
    printf("sanitized run ok: %ld A* cells, bank max %d waypoints, %d threshold hits\n", total, mx, hits);
    return 0;
}
