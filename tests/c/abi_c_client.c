/*
 * abi_c_client.c — a plain C99 caller of libfognet_hip (test infrastructure):
 * what an FFI binding or a C simulator module sees of include/fognet_hip.h.
 * Built by tests/test_abi.py (gcc -std=c99 -pedantic -Werror, CPU) and run by
 * the GPU tests.  Exit 0 = every check passed; the first failed check is
 * printed and the exit status is 1.  Without a GPU, `--no-gpu` checks that
 * fognet_create refuses cleanly.
 *
 * Checks (hand-traced answers, BrokerBaseApp3.cc:267-281 and
 * ComputeBrokerApp3.cc:269-320):
 *   fognet_decide         view {10, 9.5, 9, 12}, MIPS of node 0 = 1000, req 4000:
 *                         cost busy_j + 4 -> node 2 (9 + 4);
 *                         a 300-node view (mapped-memory path) whose minimum is node 299;
 *                         n = 0 -> FOGNET_ERR_NO_NODES, MIPS 0 -> FOGNET_ERR_DIV0
 *   fognet_decide_window  the same 4-node view, requests {4000, 0, 999999} -> {2, 2, 2}
 *   fognet_run_batch      one node (MIPS 1000, dl = ul = 1 ms): publishes at 1 s
 *                         (req 2000: S = 2 s) and 1.5 s (req 1000): task 0 starts at
 *                         1.001 s (status 5) and completes at 3.001 s; task 1 arrives
 *                         at 1.501 s, queues (status 4), runs 3.001 s .. 4.001 s.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "fognet_hip.h"

#define CHECK(cond, ...)                             \
    do {                                             \
        if (!(cond)) {                               \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);            \
            fprintf(stderr, "\n");                   \
            return 1;                                \
        }                                            \
    } while (0)

static int run_gpu(void) {
    fognet_ctx *ctx = NULL;
    int rc = fognet_create(&ctx, 0);
    CHECK(rc == FOGNET_OK, "fognet_create: %s", fognet_status_string(rc));
    CHECK(fognet_abi_version() == FOGNET_ABI_VERSION, "ABI version %d", fognet_abi_version());

    const double busy[4] = {10.0, 9.5, 9.0, 12.0};
    const int32_t mips[4] = {1000, 4000, 3000, 2000};
    int32_t k = -1;
    rc = fognet_decide(ctx, FOGNET_POLICY_REF_V3, 4, busy, mips, 4000, &k);
    CHECK(rc == FOGNET_OK && k == 2, "decide: rc %d node %d", rc, k);

    double *big = (double *)malloc(300 * sizeof(double));
    int32_t *bigm = (int32_t *)malloc(300 * sizeof(int32_t));
    for (int j = 0; j < 300; ++j) {
        big[j] = 1000.0 - j;
        bigm[j] = 1000;
    }
    rc = fognet_decide(ctx, FOGNET_POLICY_REF_V3, 300, big, bigm, 5000, &k);
    CHECK(rc == FOGNET_OK && k == 299, "decide(300): rc %d node %d", rc, k);
    free(big);
    free(bigm);

    rc = fognet_decide(ctx, FOGNET_POLICY_REF_V3, 0, busy, mips, 4000, &k);
    CHECK(rc == FOGNET_ERR_NO_NODES, "decide(n=0): rc %d", rc);
    const int32_t mips0[2] = {0, 1000};
    rc = fognet_decide(ctx, FOGNET_POLICY_REF_V3, 2, busy, mips0, 4000, &k);
    CHECK(rc == FOGNET_ERR_DIV0, "decide(MIPS 0): rc %d", rc);

    const int32_t reqs[3] = {4000, 0, 999999};
    int32_t nodes[3] = {-1, -1, -1};
    rc = fognet_decide_window(ctx, FOGNET_POLICY_REF_V3, 4, busy, mips, 3, reqs, nodes);
    CHECK(rc == FOGNET_OK && nodes[0] == 2 && nodes[1] == 2 && nodes[2] == 2, "decide_window: rc %d %d %d %d", rc,
          nodes[0], nodes[1], nodes[2]);

    const int64_t ms = 1000000000LL, s = FOGNET_TICKS_PER_SECOND;
    const int64_t arrive[2] = {1 * s, 1 * s + 500 * ms};
    const int32_t req[2] = {2000, 1000};
    const int32_t nm[1] = {1000};
    const int64_t dl[1] = {ms}, ul[1] = {ms}, init[1] = {ms};
    fognet_batch_in in;
    memset(&in, 0, sizeof in);
    in.R = 1;
    in.T = 2;
    in.N = 1;
    in.policy = FOGNET_POLICY_REF_V3;
    in.arrive_tick = arrive;
    in.req_mips = req;
    in.mips = nm;
    in.dl_tick = dl;
    in.ul_tick = ul;
    in.init_adv_tick = init;
    int32_t node[2];
    uint8_t status[2];
    int64_t start[2], done[2];
    fognet_rep_stats st;
    fognet_batch_out out;
    memset(&out, 0, sizeof out);
    out.node = node;
    out.status = status;
    out.start_tick = start;
    out.done_tick = done;
    out.stats = &st;
    rc = fognet_run_batch(ctx, &in, &out);
    CHECK(rc == FOGNET_OK, "run_batch: %s (%s)", fognet_status_string(rc), fognet_last_error(ctx));
    CHECK(node[0] == 0 && node[1] == 0, "run_batch nodes %d %d", node[0], node[1]);
    CHECK(status[0] == FOGNET_TASK_STARTED && status[1] == FOGNET_TASK_QUEUED, "statuses %d %d", status[0], status[1]);
    CHECK(start[0] == s + ms && done[0] == 3 * s + ms, "task 0: %lld .. %lld", (long long)start[0], (long long)done[0]);
    CHECK(start[1] == 3 * s + ms && done[1] == 4 * s + ms, "task 1: %lld .. %lld", (long long)start[1], (long long)done[1]);
    CHECK(st.n_tasks == 2 && st.n_queued == 1 && st.n_started == 1 && st.n_qtime == 1, "stats record");
    /* queueTime = (3.001 s - 1.501 s) * 1000: raw 1.5e15 (the recorded value 1500 ms) */
    CHECK(st.queue_min_raw == 1500000000000000LL && st.queue_max_raw == st.queue_min_raw, "queueTime raw %lld",
          (long long)st.queue_min_raw);
    fognet_destroy(ctx);
    printf("abi_c_client: all checks passed\n");
    return 0;
}

int main(int argc, char **argv) {
    if (argc > 1 && strcmp(argv[1], "--no-gpu") == 0) {
        fognet_ctx *ctx = NULL;
        int rc = fognet_create(&ctx, 0);
        CHECK(rc == FOGNET_ERR_DEVICE && ctx == NULL, "fognet_create without a GPU: rc %d", rc);
        CHECK(strcmp(fognet_status_string(FOGNET_ERR_DIV0), "advertised MIPS of node 0 is zero") == 0, "status string");
        printf("abi_c_client: no-GPU checks passed\n");
        return 0;
    }
    return run_gpu();
}
