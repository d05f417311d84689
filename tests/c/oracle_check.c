/*
 * oracle_check.c — drives the CPU restatement (oracle/, test infrastructure)
 * through every code path on synthetic traces, for the AddressSanitizer /
 * UBSan build (`make asan`).  Exit 0 when every run completed and its basic
 * invariants hold; the sanitizers abort on the first memory error or UB.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/fognet_oracle.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t next_u32(void) {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}

#define CHECK(c)                                                       \
    do {                                                               \
        if (!(c)) {                                                    \
            fprintf(stderr, "oracle_check: %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                  \
        }                                                              \
    } while (0)

/* R replications of T tasks on N nodes; tie_heavy: coarse ticks, zero services */
static int run_case(int R, int T, int N, int policy, int energy, int user, int down, int tie_heavy, int overload) {
    const int64_t base = tie_heavy ? 100000000000LL : 1;
    int64_t *arrive = malloc(sizeof(int64_t) * R * T);
    int32_t *req = malloc(sizeof(int32_t) * R * T);
    int32_t *mips = malloc(sizeof(int32_t) * N);
    int64_t *dl = malloc(sizeof(int64_t) * N), *ul = malloc(sizeof(int64_t) * N), *init = malloc(sizeof(int64_t) * N);
    int64_t *dn = malloc(sizeof(int64_t) * N);
    double *pb = malloc(sizeof(double) * N), *pi = malloc(sizeof(double) * N);
    int64_t *uu = malloc(sizeof(int64_t) * R * T), *ud = malloc(sizeof(int64_t) * R * T);
    int64_t mx = 0;
    for (int j = 0; j < N; ++j) {
        mips[j] = 1000 * (1 + j % 4);
        dl[j] = tie_heavy ? base * (int64_t)(next_u32() % 3) : 1000000 + next_u32() % 1000000000;
        ul[j] = tie_heavy ? base * (int64_t)(next_u32() % 2) : 1000000 + next_u32() % 1000000000;
        init[j] = ul[j] + (tie_heavy ? base : 0);
        if (init[j] > mx) mx = init[j];
        pb[j] = 20.0 + j;
        pi[j] = 7.0;
        dn[j] = (down && j % 3 == 1) ? mx + 5000000000000LL * (1 + j % 5) : INT64_MAX;
    }
    for (int r = 0; r < R; ++r) {
        int64_t t = mx + 1;
        for (int i = 0; i < T; ++i) {
            const int64_t gap = tie_heavy ? base * (int64_t)(next_u32() % 4)
                                          : (overload ? 1000000000LL : 10000000000LL) * (int64_t)(1 + next_u32() % 100);
            t += gap;
            arrive[(size_t)r * T + i] = t;
            req[(size_t)r * T + i] = tie_heavy ? (int32_t)(next_u32() % 4) * 500 : 1000 + (int32_t)(next_u32() % 63001);
            uu[(size_t)r * T + i] = 1000 + next_u32() % 100000;
            ud[(size_t)r * T + i] = 1000 + next_u32() % 100000;
        }
    }
    int32_t *node = malloc(sizeof(int32_t) * R * T);
    uint8_t *status = malloc((size_t)R * T);
    int64_t *start = malloc(sizeof(int64_t) * R * T), *done = malloc(sizeof(int64_t) * R * T);
    orc_rep_stats *st = calloc((size_t)R, sizeof(orc_rep_stats));
    double *ne = malloc(sizeof(double) * R * N);
    int64_t *hist = calloc((size_t)R * ORC_HIST_METRICS * ORC_HIST_BINS, sizeof(int64_t));
    orc_user_stats *us = calloc((size_t)R, sizeof(orc_user_stats));
    orc_run_batch4(R, T, N, 0, policy, arrive, req, mips, dl, ul, init, energy ? pb : NULL, energy ? pi : NULL,
                   user ? uu : NULL, user ? ud : NULL, 1, down ? dn : NULL, node, status, start, done, st,
                   energy ? ne : NULL, hist, user ? us : NULL, 4);
    int rc = 0;
    for (int r = 0; r < R && !rc; ++r) {
        if (st[r].status != ORC_OK) rc = 1;
        if (!down && st[r].n_queued + st[r].n_started != T) rc = 1;
        if (st[r].n_qtime + st[r].n_qtime_overflow > st[r].n_queued) rc = 1;
    }
    free(arrive); free(req); free(mips); free(dl); free(ul); free(init); free(dn); free(pb); free(pi); free(uu);
    free(ud); free(node); free(status); free(start); free(done); free(st); free(ne); free(hist); free(us);
    if (rc) fprintf(stderr, "oracle_check: case R=%d T=%d N=%d policy=%d failed\n", R, T, N, policy);
    return rc;
}

static int run_v2(void) {
    enum { R = 3, T = 400, N = 5 };
    int64_t arrive[R * T];
    int32_t req[R * T], bm[R], mips[N];
    double rt[R];
    int64_t stop[R], dl[N], ul[N], fa[N];
    for (int r = 0; r < R; ++r) {
        for (int i = 0; i < T; ++i) {
            arrive[r * T + i] = 50000000000LL * (i + 1);
            req[r * T + i] = 200 + (int32_t)(next_u32() % 701);
        }
        bm[r] = 1000;
        rt[r] = 0.01;
        stop[r] = 50000000000LL * (T + 2);
    }
    for (int j = 0; j < N; ++j) {
        mips[j] = 1000;
        dl[j] = ul[j] = 1000000000LL;
        fa[j] = 20000000000LL;
    }
    int32_t node[R * T];
    uint8_t status[R * T];
    int64_t start[R * T], done[R * T];
    orc_v2_stats st[R];
    orc_v2_batch b = {R, N, 0, T, arrive, req, rt, bm, stop, mips, dl, ul, fa, node, status, start, done, st};
    orc_run_v2_batch(&b, 2);
    for (int r = 0; r < R; ++r) CHECK(st[r].status == ORC_OK && st[r].n_tasks == T);
    return 0;
}

int main(void) {
    CHECK(run_case(3, 3000, 64, ORC_POLICY_REF_V3, 0, 0, 0, 0, 0) == 0);
    CHECK(run_case(2, 2000, 256, ORC_POLICY_REF_V3, 1, 1, 0, 0, 0) == 0);
    CHECK(run_case(2, 2000, 300, ORC_POLICY_EXT_LAT, 1, 0, 0, 0, 0) == 0);
    CHECK(run_case(3, 1500, 16, ORC_POLICY_REF_V3, 0, 1, 0, 1, 0) == 0);
    CHECK(run_case(2, 2000, 8, ORC_POLICY_REF_V3, 0, 1, 1, 0, 0) == 0);
    CHECK(run_case(2, 3000, 4, ORC_POLICY_REF_V3, 1, 0, 0, 0, 1) == 0);
    CHECK(run_v2() == 0);
    int32_t k = -1;
    const double busy[3] = {1.0, 0.5, 0.5};
    const int32_t m[3] = {1000, 1000, 1000};
    CHECK(orc_decide_v3(3, busy, m, 4000, &k) == ORC_OK && k == 1);
    int64_t raw = 0;
    CHECK(orc_qtime_raw(5000000000000LL, 1000000000000LL, &raw) == 1 && raw == 4000000000000000LL);
    CHECK(orc_qtime_raw(10000000000000000LL, 0, &raw) == 0);
    printf("oracle_check: ok\n");
    return 0;
}
