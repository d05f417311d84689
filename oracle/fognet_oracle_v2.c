/*
 * fognet_oracle_v2.c — TEST INFRASTRUCTURE ONLY (see fognet_oracle.h).
 *
 * Discrete-event restatement of FogNetSim++'s v2 offload model, the modules
 * simulations/example/wirelessNet.ini:56,62 select:
 *   broker  BrokerBaseApp2   src/mqttapp/BrokerBaseApp2.cc (local MIPS pool,
 *           single RELEASERESOURCE timer, "last MIPS > node 0's" forward)
 *   node    ComputeBrokerApp2 src/mqttapp/ComputeBrokerApp2.cc (MIPS
 *           reservation for requiredTime, 10-ms advert/release timer)
 * on an OMNeT++-ordered future-event set (tick, insertion sequence), like the
 * v3 restatement in fognet_oracle.c.  Trace model: publishes at the broker
 * (QoS 1, every publish registered client), fixed per-node link latencies,
 * each node's first ADVERTISEMIPS firing given (CONNACK + 0.01 s,
 * ComputeBrokerApp2.cc:250-255).  Messages without an effect on the modelled
 * state (pubAcks to users, FognetMsgTaskAck, CONNECT/CONNACK) are not
 * scheduled: they cannot reorder the events that are.
 *
 * Deadlines are doubles as in the reference: Request.requiredTime =
 * simTime().dbl() + requiredTime, compared with simTime().dbl(); OMNeT++ 4.6
 * computes dbl() as t * 1e-12 (int64 ticks times the double scale).  That
 * rounding decides some releases.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "fognet_oracle.h"

#define TICK_SCALE 1e-12           /* SimTime::dbl(): t * dscale, scale exponent -12 */
#define ADVERT_PERIOD_TICKS 10000000000LL /* scheduleAt(simTime() + 0.01, selfMsg) (ComputeBrokerApp2.cc:219) */

enum { V2_EV_PUB = 0, V2_EV_BTIMER = 1, V2_EV_NTIMER = 2, V2_EV_TASK = 3, V2_EV_ADV = 4, V2_EV_ACK6 = 5 };
enum { V2_KIND_ADVERTISEMIPS = 1, V2_KIND_RELEASERESOURCE = 2 };

typedef struct {
    int64_t tick;
    uint64_t seq;
    int32_t type, node;
    int64_t task;     /* V2_EV_PUB / TASK / ACK6 */
    int32_t mips;     /* V2_EV_ADV payload */
    uint32_t gen;     /* timers: generation (cancelEvent) */
} v2ev_t;

typedef struct {
    v2ev_t *a;
    int64_t n, cap;
} v2heap_t;

static int v2_less(const v2ev_t *x, const v2ev_t *y) {
    return x->tick != y->tick ? x->tick < y->tick : x->seq < y->seq;
}

static int v2_push(v2heap_t *h, const v2ev_t *e) {
    if (h->n == h->cap) {
        int64_t nc = h->cap ? h->cap * 2 : 64;
        v2ev_t *na = (v2ev_t *)realloc(h->a, (size_t)nc * sizeof(v2ev_t));
        if (!na) return ORC_ERR_OOM;
        h->a = na;
        h->cap = nc;
    }
    int64_t i = h->n++;
    while (i > 0) {
        int64_t p = (i - 1) >> 1;
        if (!v2_less(e, &h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = *e;
    return ORC_OK;
}

static void v2_pop(v2heap_t *h, v2ev_t *out) {
    *out = h->a[0];
    v2ev_t last = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && v2_less(&h->a[c + 1], &h->a[c])) c++;
        if (!v2_less(&h->a[c], &last)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (h->n > 0) h->a[i] = last;
}

typedef struct {
    int32_t MIPS;          /* remaining MIPS (ComputeBrokerApp2.cc:272, :226) */
    int self_scheduled, self_kind;
    uint32_t self_gen;
    int64_t *q;            /* accepted requests, oldest first (task indices) */
    double *deadline;      /* their Request.requiredTime: now.dbl() + requiredTime (:274) */
    int64_t qh, qn, qcap;
} v2node_t;

typedef struct {
    const orc_v2_in *in;
    orc_v2_out *out;
    v2heap_t fes;
    uint64_t seq;
    int64_t now;
    /* broker (BrokerBaseApp2 members) */
    int32_t MIPS;          /* own remaining MIPS (:40, :211, :386) */
    int32_t *view;         /* brokers[j]->getMips() (:128-136) */
    int b_scheduled;
    uint32_t b_gen;
    /* broker `requests` vector: tasks in insertion order with lazy erasure */
    int64_t *req_task;
    uint8_t *req_alive;    /* 0 erased, 1 local request, 2 forwarded request */
    int64_t req_h, req_n;
    int64_t *req_slot;     /* task -> its slot in req_task (-1: none) */
    v2node_t *nodes;
} v2sim_t;

static double dbl(int64_t t) { return (double)t * TICK_SCALE; }

static int64_t rt_ticks(const orc_v2_in *in) {
    /* SimTime + double: the double is converted to ticks (exact for whole
     * multiples of 1e-12 s such as the reference's 0.01 s) */
    double x = in->required_time * 1e12;
    return (int64_t)(x + (x >= 0 ? 0.5 : -0.5));
}

static int v2_schedule(v2sim_t *s, v2ev_t *e) {
    e->seq = s->seq++;
    return v2_push(&s->fes, e);
}

static int node_timer(v2sim_t *s, int32_t j, int64_t tick) {
    v2ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = tick;
    e.type = V2_EV_NTIMER;
    e.node = j;
    e.gen = s->nodes[j].self_gen;
    s->nodes[j].self_scheduled = 1;
    return v2_schedule(s, &e);
}

static int to_broker(v2sim_t *s, int32_t j, int type, int64_t task, int32_t mips) {
    v2ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = s->now + s->in->ul_tick[j];
    e.type = type;
    e.node = j;
    e.task = task;
    e.mips = mips;
    return v2_schedule(s, &e);
}

/* ComputeBrokerApp2::advertiseMIPS (:202-220): advert, then the same selfMsg
 * again 0.01 s later (its kind is left as it was). */
static int node_advertise(v2sim_t *s, int32_t j) {
    int rc = to_broker(s, j, V2_EV_ADV, -1, s->nodes[j].MIPS);
    if (rc) return rc;
    return node_timer(s, j, s->now + ADVERT_PERIOD_TICKS);
}

/* ComputeBrokerApp2::releaseResource (:222-245): the first request whose
 * deadline is strictly before now is released (one per firing), acked with
 * status 6 to the broker; then advertiseMIPS. */
static int node_release(v2sim_t *s, int32_t j) {
    v2node_t *nd = &s->nodes[j];
    double now = dbl(s->now);
    /* deadlines are nondecreasing in request order (one requiredTime per
     * trace), so the first expired request is the oldest one if any */
    if (nd->qn > 0 && nd->deadline[nd->qh] < now) {
        int64_t t = nd->q[nd->qh];
        nd->MIPS += s->in->req_mips[t];
        if (s->out->done_tick) s->out->done_tick[t] = s->now;
        s->out->stats->n_released_node++;
        nd->qh = (nd->qh + 1) % nd->qcap;
        nd->qn--;
        int rc = to_broker(s, j, V2_EV_ACK6, t, 0);
        if (rc) return rc;
    }
    return node_advertise(s, j);
}

/* ComputeBrokerApp2::processPacket, FognetMsgTask branch (:258-318). */
static int node_task(v2sim_t *s, int32_t j, int64_t t) {
    v2node_t *nd = &s->nodes[j];
    int32_t req = s->in->req_mips[t];
    if (req < nd->MIPS) { /* :269 */
        nd->MIPS -= req;  /* :272 */
        if (nd->qn == nd->qcap) {
            int64_t nc = nd->qcap ? nd->qcap * 2 : 16;
            int64_t *nq = (int64_t *)malloc((size_t)nc * sizeof(int64_t));
            double *ndl = (double *)malloc((size_t)nc * sizeof(double));
            if (!nq || !ndl) {
                free(nq);
                free(ndl);
                return ORC_ERR_OOM;
            }
            for (int64_t i = 0; i < nd->qn; i++) {
                nq[i] = nd->q[(nd->qh + i) % nd->qcap];
                ndl[i] = nd->deadline[(nd->qh + i) % nd->qcap];
            }
            free(nd->q);
            free(nd->deadline);
            nd->q = nq;
            nd->deadline = ndl;
            nd->qh = 0;
            nd->qcap = nc;
        }
        int64_t slot = (nd->qh + nd->qn) % nd->qcap;
        nd->q[slot] = t;
        nd->deadline[slot] = dbl(s->now) + s->in->required_time; /* :274 */
        nd->qn++;
        if (s->out->status) s->out->status[t] = ORC_V2_ST_ACCEPTED;
        if (s->out->start_tick) s->out->start_tick[t] = s->now;
        s->out->stats->n_accepted++;
        /* TaskAck(true) to the broker (ignored there, :139-141); cancelEvent + RELEASERESOURCE (:292-295) */
        if (nd->self_scheduled) {
            nd->self_scheduled = 0;
            nd->self_gen++;
        }
        nd->self_kind = V2_KIND_RELEASERESOURCE;
        return node_timer(s, j, s->now + rt_ticks(s->in));
    }
    if (s->out->status) s->out->status[t] = ORC_V2_ST_REJECTED; /* TaskAck(false), :299-306 */
    s->out->stats->n_rejected++;
    return ORC_OK;
}

static void broker_list_push(v2sim_t *s, int64_t t, int forwarded) {
    s->req_slot[t] = s->req_n;
    s->req_task[s->req_n] = t;
    s->req_alive[s->req_n] = forwarded ? 2 : 1;
    s->req_n++;
}

/* BrokerBaseApp2::handleMessageWhenUp, MqttMsgPublish branch (:176-195) +
 * sendPubAck (:205-287). */
static int broker_publish(v2sim_t *s, int64_t t) {
    const orc_v2_in *in = s->in;
    int32_t req = in->req_mips[t];
    s->out->stats->n_tasks++;
    int32_t k = -1, action = 0;
    orc_decide_v2(in->n_nodes, s->view, s->MIPS, req, &k, &action);
    if (s->out->node) s->out->node[t] = k;
    if (action == ORC_V2_LOCAL) { /* sendPubAck(true), :209-232 */
        s->MIPS -= req;           /* :211 */
        broker_list_push(s, t, 0); /* :212-217, deadline simTime().dbl() + requiredTime */
        if (s->out->status) s->out->status[t] = ORC_V2_ST_LOCAL;
        if (s->out->start_tick) s->out->start_tick[t] = s->now;
        s->out->stats->n_local++;
        if (s->b_scheduled) { /* cancelEvent(selfMsg) (:226) */
            s->b_scheduled = 0;
            s->b_gen++;
        }
        v2ev_t e;
        memset(&e, 0, sizeof e);
        e.tick = s->now + rt_ticks(in); /* scheduleAt(simTime() + requiredTime) (:229) */
        e.type = V2_EV_BTIMER;
        e.gen = s->b_gen;
        s->b_scheduled = 1;
        return v2_schedule(s, &e);
    }
    if (action == ORC_V2_NO_NODES) { /* :273-285: scheduleAt without cancelEvent */
        if (s->out->status) s->out->status[t] = ORC_V2_ST_NO_NODES;
        s->out->stats->n_no_nodes++;
        if (s->b_scheduled) return ORC_ERR_STATE; /* "scheduleAt(): message already scheduled" */
        v2ev_t e;
        memset(&e, 0, sizeof e);
        e.tick = s->now + rt_ticks(in);
        e.type = V2_EV_BTIMER;
        e.gen = s->b_gen;
        s->b_scheduled = 1;
        return v2_schedule(s, &e);
    }
    broker_list_push(s, t, 1); /* :255-260, before the MIPS check */
    if (action == ORC_V2_DROPPED) {
        if (s->out->status) s->out->status[t] = ORC_V2_ST_DROPPED;
        s->out->stats->n_dropped++;
        return ORC_OK;
    }
    s->out->stats->n_forwarded++;
    if (s->out->status) s->out->status[t] = ORC_V2_ST_FORWARDED; /* until the node accepts or rejects it */
    v2ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = s->now + in->dl_tick[k]; /* socket.sendTo(tsk, broker k) (:269) */
    e.type = V2_EV_TASK;
    e.node = k;
    e.task = t;
    return v2_schedule(s, &e);
}

/* BrokerBaseApp2::releaseResource (:382-406): the first request (local or
 * forwarded) whose deadline is <= now is released into the broker's own pool. */
static void broker_release(v2sim_t *s) {
    double now = dbl(s->now);
    while (s->req_h < s->req_n && !s->req_alive[s->req_h]) s->req_h++;
    if (s->req_h >= s->req_n) return;
    int64_t t = s->req_task[s->req_h];
    double deadline = dbl(s->in->arrive_tick[t]) + s->in->required_time;
    if (deadline <= now) { /* :385 (deadlines are nondecreasing in list order) */
        s->MIPS += s->in->req_mips[t]; /* :386 */
        s->out->stats->n_released_broker++;
        if (s->req_alive[s->req_h] == 2)
            s->out->stats->n_inflated++; /* a forwarded request credited to the broker's own pool */
        else if (s->out->done_tick)
            s->out->done_tick[t] = s->now;
        s->req_alive[s->req_h] = 0; /* :396 */
    }
}

static int v2_dispatch(v2sim_t *s, const v2ev_t *e) {
    s->now = e->tick;
    switch (e->type) {
    case V2_EV_PUB:
        s->out->stats->events++;
        return broker_publish(s, e->task);
    case V2_EV_BTIMER:
        if (e->gen != s->b_gen || !s->b_scheduled) return ORC_OK; /* cancelled */
        s->out->stats->events++;
        s->b_scheduled = 0;
        broker_release(s);
        return ORC_OK;
    case V2_EV_NTIMER: {
        v2node_t *nd = &s->nodes[e->node];
        if (e->gen != nd->self_gen || !nd->self_scheduled) return ORC_OK;
        s->out->stats->events++;
        nd->self_scheduled = 0;
        /* ComputeBrokerApp2::handleMessageWhenUp (:52-90) */
        if (nd->self_kind == V2_KIND_RELEASERESOURCE) return node_release(s, e->node);
        return node_advertise(s, e->node);
    }
    case V2_EV_TASK:
        s->out->stats->events++;
        return node_task(s, e->node, e->task);
    case V2_EV_ADV:
        s->out->stats->events++;
        s->view[e->node] = e->mips; /* :128-136 */
        return ORC_OK;
    case V2_EV_ACK6: {
        s->out->stats->events++;
        /* MqttMsgPuback status 6 (:143-154): relay and erase the request if it
         * is still in the list (the broker's own timer may have released it) */
        int64_t slot = s->req_slot[e->task];
        if (slot >= 0 && s->req_alive[slot]) {
            s->req_alive[slot] = 0;
            s->out->stats->n_relayed++;
        }
        return ORC_OK;
    }
    }
    return ORC_ERR_ARG;
}

int orc_run_v2_rep(const orc_v2_in *in, orc_v2_out *out) {
    v2sim_t s;
    memset(&s, 0, sizeof s);
    s.in = in;
    s.out = out;
    int32_t N = in->n_nodes;
    int64_t T = in->n_tasks;
    memset(out->stats, 0, sizeof *out->stats);
    int rc = ORC_OK;
    for (int64_t t = 0; t < T; t++) {
        if (out->node) out->node[t] = -1;
        if (out->status) out->status[t] = 0;
        if (out->start_tick) out->start_tick[t] = -1;
        if (out->done_tick) out->done_tick[t] = -1;
    }
    s.MIPS = in->broker_mips;
    s.view = (int32_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(int32_t)); /* Broker(…, MIPS 0) (:105) */
    s.nodes = (v2node_t *)calloc((size_t)(N > 0 ? N : 1), sizeof(v2node_t));
    s.req_task = (int64_t *)malloc((size_t)(T > 0 ? T : 1) * sizeof(int64_t));
    s.req_alive = (uint8_t *)calloc((size_t)(T > 0 ? T : 1), 1);
    s.req_slot = (int64_t *)malloc((size_t)(T > 0 ? T : 1) * sizeof(int64_t));
    if (!s.view || !s.nodes || !s.req_task || !s.req_alive || !s.req_slot) {
        rc = ORC_ERR_OOM;
        goto done;
    }
    for (int64_t t = 0; t < T; t++) s.req_slot[t] = -1;
    for (int32_t j = 0; j < N; j++) {
        s.nodes[j].MIPS = in->mips[j];
        s.nodes[j].self_kind = V2_KIND_ADVERTISEMIPS;
        rc = node_timer(&s, j, in->first_adv_tick[j]); /* pre-inserted, node order */
        if (rc) goto done;
    }
    for (int64_t t = 1; t < T; t++)
        if (in->arrive_tick[t] < in->arrive_tick[t - 1]) {
            rc = ORC_ERR_ARG;
            goto done;
        }
    {
        /* publishes carry the pre-insertion sequence numbers N .. N+T-1 */
        uint64_t base = s.seq;
        s.seq += (uint64_t)T;
        int64_t next = 0;
        for (;;) {
            v2ev_t e;
            int take_trace = 0;
            if (next < T) {
                if (s.fes.n == 0) {
                    take_trace = 1;
                } else {
                    v2ev_t tr;
                    tr.tick = in->arrive_tick[next];
                    tr.seq = base + (uint64_t)next;
                    take_trace = v2_less(&tr, &s.fes.a[0]);
                }
            } else if (s.fes.n == 0) {
                break;
            }
            if (take_trace) {
                memset(&e, 0, sizeof e);
                e.tick = in->arrive_tick[next];
                e.seq = base + (uint64_t)next;
                e.type = V2_EV_PUB;
                e.task = next;
            } else {
                e = s.fes.a[0];
            }
            if (e.tick >= in->stop_tick) break; /* sim-time-limit */
            if (take_trace)
                next++;
            else
                v2_pop(&s.fes, &e);
            rc = v2_dispatch(&s, &e);
            if (rc) goto done;
        }
    }
done:
    out->stats->status = rc;
    out->stats->broker_mips_final = s.MIPS;
    if (s.nodes) {
        for (int32_t j = 0; j < N; j++) {
            out->stats->node_mips_final_sum += s.nodes[j].MIPS;
            free(s.nodes[j].q);
            free(s.nodes[j].deadline);
        }
    }
    free(s.nodes);
    free(s.view);
    free(s.req_task);
    free(s.req_alive);
    free(s.req_slot);
    free(s.fes.a);
    return rc;
}

/* ---------------------------------------------------------------- batch driver */

typedef struct {
    const orc_v2_batch *b;
    int64_t next;
    pthread_mutex_t mu;
} v2batch_t;

static void *v2_worker(void *arg) {
    v2batch_t *w = (v2batch_t *)arg;
    const orc_v2_batch *b = w->b;
    for (;;) {
        pthread_mutex_lock(&w->mu);
        int64_t r = w->next++;
        pthread_mutex_unlock(&w->mu);
        if (r >= b->R) break;
        size_t to = (size_t)r * (size_t)b->T, no = (size_t)r * (size_t)b->node_stride;
        orc_v2_in in = {b->N, b->T, b->arrive_tick + to, b->req_mips + to, b->required_time[r], b->broker_mips[r],
                        b->mips + no, b->dl_tick + no, b->ul_tick + no, b->first_adv_tick + no, b->stop_tick[r]};
        orc_v2_out out = {b->node ? b->node + to : 0, b->status ? b->status + to : 0,
                          b->start_tick ? b->start_tick + to : 0, b->done_tick ? b->done_tick + to : 0, b->stats + r};
        orc_run_v2_rep(&in, &out);
    }
    return 0;
}

int orc_run_v2_batch(const orc_v2_batch *b, int threads) {
    v2batch_t w;
    w.b = b;
    w.next = 0;
    pthread_mutex_init(&w.mu, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], 0, v2_worker, &w);
    for (int i = 0; i < threads; i++) pthread_join(th[i], 0);
    pthread_mutex_destroy(&w.mu);
    return ORC_OK;
}
