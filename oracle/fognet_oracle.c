/*
 * fognet_oracle.c — TEST INFRASTRUCTURE ONLY (see fognet_oracle.h).
 *
 * A literal discrete-event restatement of the FogNetSim++ v3 offload path:
 * every reference handler on the path is one function below, and events are
 * dispatched from a future-event set ordered exactly like the OMNeT++ 4.6
 * sequential kernel orders it: (arrival tick, scheduling priority = 0,
 * insertion sequence).  Time is OMNeT++'s raw int64 simtime_t at the default
 * scale of 1e-12 s ("ticks").
 *
 * Trace-replay model: the user side and INET are
 * replaced by a pre-generated trace of publish arrivals at the broker and by
 * fixed per-node link latencies.  Trace publishes and each node's initial
 * ADVERTISEMIPS self-message are inserted into the FES before the run starts
 * (nodes first, then publishes in trace order); everything else is inserted
 * when the reference code would call scheduleAt()/sendTo().
 */
#include "fognet_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define TICKS_PER_SECOND 1000000000000LL /* simtime scale 1e-12 (no simtime-scale in any ini) */

enum { EV_PUBLISH = 0, EV_ADVERT = 1, EV_TASK = 2, EV_SELF = 3, EV_ACK_AT_BROKER = 4, EV_ACK_AT_USER = 5, EV_CRASH = 6 };
enum { KIND_ADVERTISEMIPS = 1, KIND_RELEASERESOURCE = 2 }; /* ComputeBrokerApp3.h selfMsg kinds */
/* internal: the reference run ended at a queueTime throw (stop_at_ref_abort) */
#define ORC_STOPPED (-100)

typedef struct {
    int64_t tick;
    uint64_t seq;
    int32_t type;
    int32_t node;
    int64_t task;
    int32_t mips;    /* EV_ADVERT payload: FognetMsgAdvertiseMIPS.MIPS; EV_ACK_*: MqttMsgPuback.status */
    uint32_t gen;    /* EV_SELF: selfMsg generation (cancelEvent support)  */
    double busy;     /* EV_ADVERT payload: FognetMsgAdvertiseMIPS.busyTime */
} ev_t;

typedef struct {
    ev_t *a;
    int64_t n, cap;
} heap_t;

static int ev_less(const ev_t *x, const ev_t *y) {
    if (x->tick != y->tick) return x->tick < y->tick;
    return x->seq < y->seq;
}

static int heap_push(heap_t *h, const ev_t *e) {
    if (h->n == h->cap) {
        int64_t nc = h->cap ? h->cap * 2 : 256;
        ev_t *na = (ev_t *)realloc(h->a, (size_t)nc * sizeof(ev_t));
        if (!na) return ORC_ERR_OOM;
        h->a = na;
        h->cap = nc;
    }
    int64_t i = h->n++;
    while (i > 0) {
        int64_t p = (i - 1) >> 1;
        if (!ev_less(e, &h->a[p])) break;
        h->a[i] = h->a[p];
        i = p;
    }
    h->a[i] = *e;
    return ORC_OK;
}

static void heap_pop(heap_t *h, ev_t *out) {
    *out = h->a[0];
    ev_t last = h->a[--h->n];
    int64_t i = 0;
    for (;;) {
        int64_t c = 2 * i + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && ev_less(&h->a[c + 1], &h->a[c])) c++;
        if (!ev_less(&h->a[c], &last)) break;
        h->a[i] = h->a[c];
        i = c;
    }
    if (h->n > 0) h->a[i] = last;
}

/* Request record as the node keeps it (Request.cc:34-48; queueStartTime :25). */
typedef struct {
    int64_t task;
    double required_time; /* tskTime, seconds (integer-valued) */
    int64_t qstart_tick;  /* queueStartTime (ComputeBrokerApp3.cc:306) */
} req_t;

/* One fog node: ComputeBrokerApp3 members (ComputeBrokerApp3.h). */
typedef struct {
    int32_t MIPS;
    double busyTime;       /* ComputeBrokerApp3.cc:46 */
    int resourceStatus;    /* false = idle */
    req_t currentTask;
    int self_scheduled;    /* selfMsg->isScheduled() */
    int self_kind;         /* selfMsg->getKind()     */
    uint32_t self_gen;
    req_t *q;              /* FIFO `requests` (push_back / erase(begin)) */
    int64_t qh, qn, qcap;
    int64_t pending;       /* assigned by the broker, advert of its completion not yet at broker */
    int64_t served_s;      /* service seconds of completed tasks (energy model, a11) */
    int down;              /* crashed (node-down extension): the app handles nothing */
} node_t;

typedef struct {
    const orc_rep_in *in;
    orc_rep_out *out;
    heap_t fes;
    uint64_t seq;
    int64_t now;
    /* broker: BrokerBaseApp3 `brokers` vector (Broker.cc:21-22) */
    double *adv_busy;
    int32_t *adv_mips;
    node_t *nodes;
    orc_rep_stats st;
} sim_t;

static void acc128(uint64_t *lo, uint64_t *hi, uint64_t v_lo, uint64_t v_hi) {
    uint64_t o = *lo;
    *lo += v_lo;
    *hi += v_hi + (*lo < o);
}

static void acc_moment(uint64_t *sum_lo, uint64_t *sum_hi, uint64_t *sq_lo, uint64_t *sq_hi, int64_t v) {
    /* v >= 0 for response times */
    unsigned __int128 sq = (unsigned __int128)(uint64_t)v * (uint64_t)v;
    acc128(sum_lo, sum_hi, (uint64_t)v, 0);
    acc128(sq_lo, sq_hi, (uint64_t)sq, (uint64_t)(sq >> 64));
}

/* signed value: two's complement 128-bit sum, 192-bit sum of squares */
static void acc_moment_signed(uint64_t *sum_lo, uint64_t *sum_hi, uint64_t *sq_lo, uint64_t *sq_hi,
                              uint64_t *sq_top, int64_t v) {
    uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    unsigned __int128 sq = (unsigned __int128)m * m;
    acc128(sum_lo, sum_hi, (uint64_t)v, v < 0 ? ~(uint64_t)0 : 0);
    unsigned __int128 q = ((unsigned __int128)*sq_hi << 64) | *sq_lo;
    unsigned __int128 n = q + sq;
    *sq_lo = (uint64_t)n;
    *sq_hi = (uint64_t)(n >> 64);
    *sq_top += n < q; /* carry out of bit 127 */
}

int orc_hist_bin(int64_t ticks) {
    /* fognet_hip.h FOGNET_HIST_BINS: whole milliseconds, log2 bins */
    uint64_t q = (uint64_t)ticks / 1000000000ull;
    if (ticks < 0 || q == 0) return 0;
    int b = 64 - __builtin_clzll(q);
    return b > ORC_HIST_BINS - 1 ? ORC_HIST_BINS - 1 : b;
}

/* ---- OMNeT++ 4.6 SimTime arithmetic (fognet_oracle.h) */

static double simtime_dbl(int64_t t) { return (double)t * 1e-12; } /* dbl() = t * invfscale */

static int simtime_toint64(double x, int64_t *out) { /* SimTime::toInt64 */
    double f = floor(x + 0.5);
    if (!(fabs(f) < 9223372036854775808.0)) return 0; /* cRuntimeError: out of range */
    *out = (int64_t)f;
    return 1;
}

int orc_qtime_raw(int64_t now, int64_t qstart, int64_t *raw) {
    int64_t qs = 0;
    simtime_toint64(1e12 * simtime_dbl(qstart), &qs); /* simTime() - (double)queueStartTime: SimTime(double) */
    return simtime_toint64((double)(now - qs) * 1000.0, raw); /* ... * 1000 (ComputeBrokerApp3.cc:238) */
}

int orc_ms_raw(int64_t diff_ticks, int64_t *raw) { return simtime_toint64((double)diff_ticks * 1000.0, raw); }

int orc_hist_bin_raw(int64_t raw) {
    /* the recorded double (dbl() of the emitted value), in whole "ms" */
    double v = simtime_dbl(raw);
    if (!(v >= 1.0)) return 0;
    uint64_t q = (uint64_t)v;
    int b = 64 - __builtin_clzll(q);
    return b > ORC_HIST_BINS - 1 ? ORC_HIST_BINS - 1 : b;
}

static void hist_add(sim_t *s, int metric, int64_t ticks) {
    if (s->out->hist) s->out->hist[metric * ORC_HIST_BINS + orc_hist_bin(ticks)]++;
}

static void hist_add_raw(sim_t *s, int metric, int64_t raw) {
    if (s->out->hist) s->out->hist[metric * ORC_HIST_BINS + orc_hist_bin_raw(raw)]++;
}

static int schedule(sim_t *s, ev_t *e) {
    e->seq = s->seq++;
    return heap_push(&s->fes, e);
}

/* ---- user side (only when the trace carries user links) */

static int64_t user_ul(const sim_t *s, int64_t t) { return s->in->user_ul_tick[s->in->user_per_task ? t : 0]; }
static int64_t user_dl(const sim_t *s, int64_t t) { return s->in->user_dl_tick[s->in->user_per_task ? t : 0]; }

static void moment_add(orc_moments *m, int64_t v) {
    m->count++;
    if (v < m->min_raw) m->min_raw = v;
    if (v > m->max_raw) m->max_raw = v;
    acc_moment_signed(&m->sum_lo, &m->sum_hi, &m->sq_lo, &m->sq_hi, &m->sq_top, v);
}

/* emit(signal, (simTime() - created) * 1000): dropped when the simtime_t
 * product overflows (the cRuntimeError is swallowed by the handler's
 * catch (std::exception&), mqttApp2.cc:253,293) */
static void moment_add_ms(orc_moments *m, int64_t diff_ticks) {
    int64_t raw;
    if (orc_ms_raw(diff_ticks, &raw)) moment_add(m, raw);
    else m->overflow++;
}

/* socket.sendTo(MqttMsgPuback{status}) towards task t's user: from the broker
 * (one user downlink later at the user) or from node k (one uplink later at the
 * broker, which relays it, BrokerBaseApp3.cc:164-198). */
static int send_ack(sim_t *s, int at_broker, int32_t k, int64_t t, int32_t status) {
    if (!s->in->user_ul_tick || !s->out->user) return ORC_OK;
    ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = s->now + (at_broker ? user_dl(s, t) : s->in->ul_tick[k]);
    e.type = at_broker ? EV_ACK_AT_USER : EV_ACK_AT_BROKER;
    e.node = k;
    e.task = t;
    e.mips = status;
    return schedule(s, &e);
}

/* mqttApp2::processPacket, MqttMsgPuback branch (mqttApp2.cc:252-291): the
 * signal is (simTime() - timeCreated) * 1000, timeCreated a simtime_t (raw emitted value). */
static void user_ack(sim_t *s, const ev_t *e) {
    orc_user_stats *u = s->out->user;
    int64_t created = s->in->arrive_tick[e->task] - user_ul(s, e->task); /* sendMqttData: created at the user */
    int64_t v = s->now - created;
    if (e->mips == 5) moment_add_ms(&u->latency, v);        /* :257-265 */
    else if (e->mips == 4) moment_add_ms(&u->latencyH1, v); /* :269-277 */
    else if (e->mips == 6) moment_add_ms(&u->taskTime, v);  /* :279-291 */
}

/* The engine's simulated-time range (fognet_hip.h: every tick below 2^61, 26.7
 * days).  A RELEASERESOURCE past it is refused (ORC_ERR_ARG) like the engine
 * refuses it; it also keeps tskTime * 1e12 clear of int64 overflow. */
#define ORC_MAX_TICK ((int64_t)1 << 61)

static int release_tick(const sim_t *s, double tskTime, int64_t *tick) {
    if (!(tskTime < 4194304.0)) return ORC_ERR_ARG; /* 2^22 s > 2^61 ticks */
    *tick = s->now + (int64_t)tskTime * TICKS_PER_SECOND;
    return *tick > ORC_MAX_TICK ? ORC_ERR_ARG : ORC_OK;
}

/* cSimpleModule::scheduleAt for a node's selfMsg. */
static int node_schedule_self(sim_t *s, int32_t k, int64_t tick, int kind) {
    node_t *nd = &s->nodes[k];
    if (nd->self_scheduled) return ORC_ERR_STATE; /* "scheduleAt(): message already scheduled" */
    nd->self_scheduled = 1;
    nd->self_kind = kind;
    ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = tick;
    e.type = EV_SELF;
    e.node = k;
    e.gen = nd->self_gen;
    return schedule(s, &e);
}

/* cSimpleModule::cancelEvent(selfMsg): lazily invalidates the pending event. */
static void node_cancel_self(sim_t *s, int32_t k) {
    node_t *nd = &s->nodes[k];
    if (nd->self_scheduled) {
        nd->self_scheduled = 0;
        nd->self_gen++;
    }
}

/* ComputeBrokerApp3::advertiseMIPS, ComputeBrokerApp3.cc:205-222: the advert carries
 * {MIPS, busyTime} and is delivered to the broker one uplink latency later. */
static int node_advertise(sim_t *s, int32_t k, int64_t completed_task) {
    node_t *nd = &s->nodes[k];
    ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = s->now + s->in->ul_tick[k];
    e.type = EV_ADVERT;
    e.node = k;
    e.task = completed_task;
    e.mips = nd->MIPS;
    e.busy = nd->busyTime;
    return schedule(s, &e);
}

/* ComputeBrokerApp3::releaseResource, ComputeBrokerApp3.cc:224-256. */
static int node_release(sim_t *s, int32_t k) {
    node_t *nd = &s->nodes[k];
    int64_t t = nd->currentTask.task;
    /* ack status 6 to the broker (:228-233) -- relay only, no decision effect */
    int rc0 = send_ack(s, 0, k, t, 6);
    if (rc0) return rc0;
    nd->busyTime = nd->busyTime - nd->currentTask.required_time; /* :232 */
    nd->resourceStatus = 0;                                      /* :234 */
    nd->served_s += (int64_t)nd->currentTask.required_time;
    s->st.busy_s += (int64_t)nd->currentTask.required_time;
    if (s->out->done_tick) s->out->done_tick[t] = s->now;
    {
        int64_t resp = s->now - s->in->arrive_tick[t];
        acc_moment(&s->st.resp_sum_lo, &s->st.resp_sum_hi, &s->st.resp_sq_lo, &s->st.resp_sq_hi, resp);
        if (resp < s->st.resp_min_ticks) s->st.resp_min_ticks = resp;
        if (resp > s->st.resp_max_ticks) s->st.resp_max_ticks = resp;
        hist_add(s, 1, resp);
        if (s->now > s->st.last_tick) s->st.last_tick = s->now;
    }
    if (nd->qn > 0) { /* :236-252 */
        nd->resourceStatus = 1;
        req_t *h = &nd->q[nd->qh];
        /* emit(queueTimeSignal, (simTime() - queueStartTime) * 1000) (:238): the raw
         * emitted simtime_t; an overflow is a cRuntimeError in the reference (counted) */
        int64_t qt;
        if (orc_qtime_raw(s->now, h->qstart_tick, &qt)) {
            acc_moment_signed(&s->st.queue_sum_lo, &s->st.queue_sum_hi, &s->st.queue_sq_lo, &s->st.queue_sq_hi,
                              &s->st.queue_sq_top, qt);
            if (qt < s->st.queue_min_raw) s->st.queue_min_raw = qt;
            if (qt > s->st.queue_max_raw) s->st.queue_max_raw = qt;
            s->st.n_qtime++;
            hist_add_raw(s, 0, qt);
        } else {
            /* cRuntimeError out of emit(): nothing catches it before the kernel
             * (:84-86), the reference run ends here.  Events come in tick order, so the
             * first overflow has the abort tick; at that tick the lowest task index. */
            s->st.n_qtime_overflow++;
            if (s->now < s->st.abort_tick || (s->now == s->st.abort_tick && h->task < s->st.abort_task)) {
                s->st.abort_tick = s->now;
                s->st.abort_task = h->task;
            }
            if (s->in->stop_at_ref_abort) return ORC_STOPPED;
        }
        nd->currentTask = *h; /* :240-244 */
        nd->qh = (nd->qh + 1) % nd->qcap; /* requests.erase(begin) (:246) */
        nd->qn--;
        if (s->out->start_tick) s->out->start_tick[nd->currentTask.task] = s->now;
        node_cancel_self(s, k); /* :248-249 */
        int64_t at;
        int rc = release_tick(s, nd->currentTask.required_time, &at);
        if (rc) return rc;
        rc = node_schedule_self(s, k, at, KIND_RELEASERESOURCE); /* :250 */
        if (rc) return rc;
    }
    return node_advertise(s, k, t); /* :254 */
}

/* ComputeBrokerApp3::processPacket, FognetMsgTask branch, ComputeBrokerApp3.cc:269-320. */
static int node_task(sim_t *s, int32_t k, int64_t t) {
    node_t *nd = &s->nodes[k];
    if (nd->down) { /* a crashed host drops the packet: no ack, no service */
        if (s->out->status) s->out->status[t] = ORC_TASK_LOST;
        return ORC_OK;
    }
    int32_t req = s->in->req_mips[t];
    if (nd->MIPS == 0) return ORC_ERR_DIV0;
    double tskTime = (double)(req / nd->MIPS); /* :276 int / int */
    nd->busyTime = nd->busyTime + tskTime;     /* :279 */
    if (nd->resourceStatus == 0) {             /* :282 */
        nd->resourceStatus = 1;
        if (s->out->status) s->out->status[t] = 5; /* "task assigned" (:285-289) */
        int rc5 = send_ack(s, 0, k, t, 5);
        if (rc5) return rc5;
        nd->currentTask.task = t;
        nd->currentTask.required_time = tskTime; /* :292-296 */
        nd->currentTask.qstart_tick = s->now;
        if (s->out->start_tick) s->out->start_tick[t] = s->now;
        s->st.n_started++;
        int64_t at;
        int rc = release_tick(s, tskTime, &at);
        if (rc) return rc;
        return node_schedule_self(s, k, at, KIND_RELEASERESOURCE); /* :299-301, no cancelEvent */
    }
    /* busy: FIFO enqueue (:305-309), ack status 4 "task queued" (:310-313) */
    if (nd->qn == nd->qcap) {
        int64_t nc = nd->qcap ? nd->qcap * 2 : 16;
        req_t *nq = (req_t *)malloc((size_t)nc * sizeof(req_t));
        if (!nq) return ORC_ERR_OOM;
        for (int64_t i = 0; i < nd->qn; i++) nq[i] = nd->q[(nd->qh + i) % nd->qcap];
        free(nd->q);
        nd->q = nq;
        nd->qh = 0;
        nd->qcap = nc;
    }
    req_t *r = &nd->q[(nd->qh + nd->qn) % nd->qcap];
    r->task = t;
    r->required_time = tskTime;
    r->qstart_tick = s->now;
    nd->qn++;
    if (s->out->status) s->out->status[t] = 4;
    s->st.n_queued++;
    return send_ack(s, 0, k, t, 4);
}

int orc_decide_v3(int32_t n, const double *adv_busy, const int32_t *adv_mips, int32_t req, int32_t *out_node) {
    /* BrokerBaseApp3::sendPubAck, status==false branch, BrokerBaseApp3.cc:265-281 */
    if (n <= 0) return ORC_ERR_NO_NODES;    /* :268 dereferences brokers[0] first */
    if (adv_mips[0] == 0) return ORC_ERR_DIV0; /* :268 int division by brokers[0]->getMips() */
    int32_t currentGoodBroker = 0;             /* :267 */
    double tskTime = (double)(req / adv_mips[0]); /* :268 (int/int, then to double) */
    double tempp = adv_busy[0] + tskTime;         /* :270 */
    if (n > 1) {                                  /* :271 */
        for (int32_t j = 0; j < n; j++) {         /* :272 */
            if (adv_busy[j] + (double)(req / adv_mips[0]) < tempp) { /* :273 strict '<' */
                tempp = adv_busy[j] + (double)(req / adv_mips[0]);   /* :275 */
                currentGoodBroker = j;                               /* :277 */
            }
        }
    }
    *out_node = currentGoodBroker;
    return ORC_OK;
}

int orc_decide_ext_lat(int32_t n, const double *adv_busy, const int32_t *mips, const int64_t *dl, int32_t req,
                       int32_t *out_node) {
    /* Extension policy (BASELINE.json north_star cost; NOT in the reference): network
     * delay + advertised backlog + service time at the node's own MIPS, in exact uint64
     * ticks: dl_j + (busy_j + min(req / mips_j, 2^20)) * 1e12, ties -> lowest j. */
    if (n <= 0) return ORC_ERR_NO_NODES;
    int32_t best = -1;
    uint64_t best_c = 0;
    for (int32_t j = 0; j < n; j++) {
        if (mips[j] <= 0) return ORC_ERR_DIV0;
        if (dl[j] < 0 || dl[j] >= (1LL << 50)) return ORC_ERR_ARG; /* keeps the cost below 2^64 */
        uint64_t s = (uint64_t)(req / mips[j]);
        if (s > (1u << 20)) s = 1u << 20; /* saturation (fognet_hip.h), never decisive for admissible tasks */
        uint64_t c = (uint64_t)dl[j] + ((uint64_t)adv_busy[j] + s) * (uint64_t)TICKS_PER_SECOND;
        if (best < 0 || c < best_c) {
            best_c = c;
            best = j;
        }
    }
    *out_node = best;
    return ORC_OK;
}

int orc_decide_hier(int32_t n, const double *adv_busy, const int32_t *adv_mips, int32_t region, int32_t threshold_s,
                    int32_t req, int32_t *out_node, int32_t *escalated) {
    /* Extension (fognet_hip.h FOGNET_POLICY_EXT_HIER; not in the reference): the regional
     * broker runs BrokerBaseApp3's rule (BrokerBaseApp3.cc:267-281) over its own node list,
     * nodes region*1024 .. region*1024+1023, and escalates to the parent, which runs it over
     * every node, when its choice's advertised busy time exceeds the threshold. */
    int32_t lo = region * ORC_HIER_REGION_NODES, hi = lo + ORC_HIER_REGION_NODES;
    if (region < 0 || lo >= n) return ORC_ERR_ARG;
    if (hi > n) hi = n;
    int32_t k;
    int rc = orc_decide_v3(hi - lo, adv_busy + lo, adv_mips + lo, req, &k);
    if (rc) return rc;
    k += lo;
    *escalated = adv_busy[k] > (double)threshold_s;
    if (*escalated) {
        rc = orc_decide_v3(n, adv_busy, adv_mips, req, &k);
        if (rc) return rc;
    }
    *out_node = k;
    return ORC_OK;
}

int orc_decide_v2(int32_t n, const int32_t *adv_mips, int32_t local_mips, int32_t req, int32_t *out_node,
                  int32_t *out_action) {
    /* BrokerBaseApp2::handleMessageWhenUp, MqttMsgPublish branch (BrokerBaseApp2.cc:180-192) */
    if (req < local_mips) { /* :181 */
        *out_node = -1;
        *out_action = ORC_V2_LOCAL;
        return ORC_OK;
    }
    /* sendPubAck(..., false), :235-286 */
    if (n <= 0) { /* :239, :273-285 */
        *out_node = -1;
        *out_action = ORC_V2_NO_NODES;
        return ORC_OK;
    }
    int32_t currentGoodBroker = 0;      /* :237 */
    int32_t temp = adv_mips[0];         /* :241 */
    for (int32_t i = 0; i < n; i++) {   /* :242 */
        if (i + 1 < n) {                /* :243 */
            if (adv_mips[i + 1] > temp) /* :244, temp never updated */
                currentGoodBroker = i + 1;
        }
    }
    *out_node = currentGoodBroker;
    *out_action = req < adv_mips[currentGoodBroker] ? ORC_V2_FORWARD : ORC_V2_DROPPED; /* :262 */
    return ORC_OK;
}

/* BrokerBaseApp3::handleMessageWhenUp, MqttMsgPublish branch (:138-158) + sendPubAck(false). */
static int broker_publish(sim_t *s, int64_t t) {
    /* QoS==1 in every trace publish; the status-4 pubAck to the user (:145-150) and the
     * `delay` emit (:143) do not influence the decision. */
    int32_t k;
    int rc;
    if (s->in->user_ul_tick && s->out->user) {
        moment_add(&s->out->user->delay, user_ul(s, t)); /* emit(delaySignal, simTime() - creationTime) (:143) */
        rc = send_ack(s, 1, -1, t, 4);                    /* pubAck status 4 (:145-150) */
        if (rc) return rc;
    }
    int32_t escalated = 0;
    if (s->in->policy == ORC_POLICY_EXT_LAT)
        rc = orc_decide_ext_lat(s->in->n_nodes, s->adv_busy, s->in->mips, s->in->dl_tick, s->in->req_mips[t], &k);
    else if (s->in->policy == ORC_POLICY_EXT_HIER)
        rc = orc_decide_hier(s->in->n_nodes, s->adv_busy, s->adv_mips, s->in->region ? s->in->region[t] : -1,
                             s->in->hier_threshold_s, s->in->req_mips[t], &k, &escalated);
    else
        rc = orc_decide_v3(s->in->n_nodes, s->adv_busy, s->adv_mips, s->in->req_mips[t], &k);
    if (rc) return rc;
    if (s->out->node) s->out->node[t] = k;
    s->st.n_tasks++;
    node_t *nd = &s->nodes[k];
    nd->pending++;
    if (nd->pending > s->st.max_pending) s->st.max_pending = (int32_t)nd->pending;
    /* socket.sendTo(tsk, brokers[k]) (:302): delivered one downlink latency later (an escalated
     * task first takes the regional -> parent hop) */
    ev_t e;
    memset(&e, 0, sizeof e);
    e.tick = s->now + s->in->dl_tick[k] + (escalated ? s->in->hier_up_tick : 0);
    e.type = EV_TASK;
    e.node = k;
    e.task = t;
    return schedule(s, &e);
}

/* BrokerBaseApp3::handleMessageWhenUp, FognetMsgAdvertiseMIPS branch (:123-130). */
static void broker_advert(sim_t *s, const ev_t *e) {
    s->adv_mips[e->node] = e->mips;  /* setMips   (:127) */
    s->adv_busy[e->node] = e->busy;  /* setBusyTime (:128) */
}

static int dispatch(sim_t *s, const ev_t *e) {
    s->now = e->tick;
    if (e->type == EV_ACK_AT_BROKER) /* relay to the request's user (BrokerBaseApp3.cc:164-198) */
        return send_ack(s, 1, e->node, e->task, e->mips);
    if (e->type == EV_ACK_AT_USER) {
        user_ack(s, e);
        return ORC_OK;
    }
    if (e->type == EV_CRASH) { /* handleNodeCrash: cancelEvent(selfMsg) (ComputeBrokerApp3.cc:423-427) */
        s->nodes[e->node].down = 1;
        node_cancel_self(s, e->node);
        return ORC_OK;
    }
    if (e->type == EV_SELF && (e->gen != s->nodes[e->node].self_gen || !s->nodes[e->node].self_scheduled))
        return ORC_OK; /* cancelled: cancelEvent removed it from the FES, not an event */
    s->st.events++;
    switch (e->type) {
    case EV_PUBLISH:
        return broker_publish(s, e->task);
    case EV_ADVERT:
        broker_advert(s, e);
        if (e->task >= 0) s->nodes[e->node].pending--; /* completion adverts only */
        return ORC_OK;
    case EV_TASK:
        return node_task(s, e->node, e->task);
    case EV_SELF: {
        node_t *nd = &s->nodes[e->node];
        if (e->gen != nd->self_gen || !nd->self_scheduled) return ORC_OK; /* cancelled */
        nd->self_scheduled = 0;
        /* ComputeBrokerApp3::handleMessageWhenUp self-message switch (:65-90) */
        if (nd->self_kind == KIND_ADVERTISEMIPS) {
            /* initial advert: advertiseMIPS() with task = -1 marker */
            ev_t a;
            memset(&a, 0, sizeof a);
            a.tick = s->now + s->in->ul_tick[e->node];
            a.type = EV_ADVERT;
            a.node = e->node;
            a.task = -1;
            a.mips = nd->MIPS;
            a.busy = nd->busyTime;
            return schedule(s, &a);
        }
        return node_release(s, e->node);
    }
    }
    return ORC_ERR_ARG;
}

int orc_run_rep(const orc_rep_in *in, orc_rep_out *out) {
    sim_t s;
    memset(&s, 0, sizeof s);
    s.in = in;
    s.out = out;
    int32_t N = in->n_nodes;
    int64_t T = in->n_tasks;
    s.st.queue_min_raw = INT64_MAX;
    s.st.resp_min_ticks = INT64_MAX;
    s.st.queue_max_raw = INT64_MIN;
    s.st.resp_max_ticks = INT64_MIN;
    s.st.last_tick = INT64_MIN;
    s.st.abort_tick = INT64_MAX;
    s.st.abort_task = -1;
    if (out->user) {
        orc_moments *ms[4] = {&out->user->delay, &out->user->latency, &out->user->latencyH1, &out->user->taskTime};
        for (int i = 0; i < 4; i++) {
            memset(ms[i], 0, sizeof *ms[i]);
            ms[i]->min_raw = INT64_MAX;
            ms[i]->max_raw = INT64_MIN;
        }
    }
    int rc = ORC_OK;
    for (int64_t t = 0; t < T; t++) {
        if (out->node) out->node[t] = -1;
        if (out->start_tick) out->start_tick[t] = -1;
        if (out->done_tick) out->done_tick[t] = -1;
    }
    if (N <= 0) {
        rc = ORC_ERR_NO_NODES;
        goto done;
    }
    s.adv_busy = (double *)calloc((size_t)N, sizeof(double));
    s.adv_mips = (int32_t *)calloc((size_t)N, sizeof(int32_t));
    s.nodes = (node_t *)calloc((size_t)N, sizeof(node_t));
    if (!s.adv_busy || !s.adv_mips || !s.nodes) {
        rc = ORC_ERR_OOM;
        goto done;
    }
    for (int32_t k = 0; k < N; k++) s.nodes[k].MIPS = in->mips[k];

    /* Pre-inserted events: each node's initial ADVERTISEMIPS self-message (sent one
     * uplink latency before it reaches the broker), then every trace publish. */
    for (int32_t k = 0; k < N; k++) {
        rc = node_schedule_self(&s, k, in->init_adv_tick[k] - in->ul_tick[k], KIND_ADVERTISEMIPS);
        if (rc) goto done;
    }
    /* node-down extension: crashes are scheduled at setup, so each precedes
     * every event of its tick that is inserted later (all model events).  The
     * energy model assumes a node that is up for the whole run. */
    if (in->down_tick && in->p_busy_w) {
        rc = ORC_ERR_UNSUPPORTED;
        goto done;
    }
    if (in->down_tick)
        for (int32_t k = 0; k < N; k++) {
            if (in->down_tick[k] == INT64_MAX) continue;
            if (in->down_tick[k] < in->init_adv_tick[k]) {
                rc = ORC_ERR_ARG;
                goto done;
            }
            ev_t c;
            memset(&c, 0, sizeof c);
            c.tick = in->down_tick[k];
            c.type = EV_CRASH;
            c.node = k;
            rc = schedule(&s, &c);
            if (rc) goto done;
        }
    int sorted = 1;
    for (int64_t t = 1; t < T; t++)
        if (in->arrive_tick[t] < in->arrive_tick[t - 1]) {
            sorted = 0;
            break;
        }
    if (sorted) {
        /* Same FES order as inserting every publish up front: publish t carries
         * sequence number N + t, below every dynamically scheduled event. */
        uint64_t base = s.seq;
        s.seq += (uint64_t)T;
        int64_t next = 0;
        while (next < T || s.fes.n > 0) {
            int take_trace = 0;
            if (next < T) {
                if (s.fes.n == 0) take_trace = 1;
                else {
                    ev_t tr;
                    tr.tick = in->arrive_tick[next];
                    tr.seq = base + (uint64_t)next;
                    take_trace = ev_less(&tr, &s.fes.a[0]);
                }
            }
            ev_t e;
            if (take_trace) {
                memset(&e, 0, sizeof e);
                e.tick = in->arrive_tick[next];
                e.seq = base + (uint64_t)next;
                e.type = EV_PUBLISH;
                e.task = next++;
            } else {
                heap_pop(&s.fes, &e);
            }
            rc = dispatch(&s, &e);
            if (rc) goto done;
        }
    } else {
        for (int64_t t = 0; t < T; t++) {
            ev_t e;
            memset(&e, 0, sizeof e);
            e.tick = in->arrive_tick[t];
            e.type = EV_PUBLISH;
            e.task = t;
            rc = schedule(&s, &e);
            if (rc) goto done;
        }
        while (s.fes.n > 0) {
            ev_t e;
            heap_pop(&s.fes, &e);
            rc = dispatch(&s, &e);
            if (rc) goto done;
        }
    }
    if (out->final_view_busy)
        for (int32_t k = 0; k < N; k++) out->final_view_busy[k] = s.adv_busy[k];
    if (in->p_busy_w && in->p_idle_w) {
        /* a11 energy (builder-defined, fognet_hip.h fognet_rep_stats.energy_j) */
        int64_t H = s.st.n_tasks > 0 ? s.st.last_tick : 0;
        double e_sum = 0.0;
        for (int32_t k = 0; k < N; k++) {
            double eb = in->p_busy_w[k] * (double)s.nodes[k].served_s;
            double idle = (double)(H - s.nodes[k].served_s * TICKS_PER_SECOND) / 1e12;
            double ei = in->p_idle_w[k] * idle;
            double e = eb + ei;
            if (out->node_energy_j) out->node_energy_j[k] = e;
            e_sum = e_sum + e;
        }
        s.st.energy_j = e_sum;
    }
done:
    if (rc == ORC_STOPPED) rc = ORC_OK; /* the reference's own end of run (stop_at_ref_abort) */
    s.st.status = rc;
    if (out->stats) *out->stats = s.st;
    if (s.nodes)
        for (int32_t k = 0; k < N; k++) free(s.nodes[k].q);
    free(s.nodes);
    free(s.adv_busy);
    free(s.adv_mips);
    free(s.fes.a);
    return rc;
}

/* ---------------------------------------------------------------- batch driver */

typedef struct {
    int32_t R, N, node_stride, policy;
    int64_t T;
    const int64_t *arrive_tick;
    const int32_t *req_mips, *mips;
    const int64_t *dl, *ul, *init_adv;
    const double *p_busy, *p_idle;
    const int64_t *user_ul, *user_dl;
    int32_t user_per_task;
    const int64_t *down;
    const int32_t *region;
    int32_t hier_threshold_s;
    int64_t hier_up_tick;
    int32_t flags;
    int32_t *node;
    uint8_t *status;
    int64_t *start_tick, *done_tick;
    orc_rep_stats *stats;
    double *node_energy;
    int64_t *hist;
    orc_user_stats *user;
    int64_t next; /* work counter */
    pthread_mutex_t mu;
} batch_t;

static void *batch_worker(void *arg) {
    batch_t *b = (batch_t *)arg;
    for (;;) {
        pthread_mutex_lock(&b->mu);
        int64_t r = b->next++;
        pthread_mutex_unlock(&b->mu);
        if (r >= b->R) break;
        size_t to = (size_t)r * (size_t)b->T, no = (size_t)r * (size_t)b->node_stride;
        size_t uo = b->user_per_task ? to : (size_t)r;
        orc_rep_in in = {b->N, b->T, b->arrive_tick + to, b->req_mips + to, b->mips + no,
                         b->dl + no, b->ul + no, b->init_adv + no,
                         b->p_busy ? b->p_busy + no : 0, b->p_idle ? b->p_idle + no : 0, b->policy,
                         b->user_ul ? b->user_ul + uo : 0, b->user_dl ? b->user_dl + uo : 0, b->user_per_task,
                         b->down ? b->down + no : 0, b->region ? b->region + to : 0, b->hier_threshold_s,
                         b->hier_up_tick, b->flags & 1};
        orc_rep_out out = {b->node ? b->node + to : 0, b->status ? b->status + to : 0,
                           b->start_tick ? b->start_tick + to : 0, b->done_tick ? b->done_tick + to : 0,
                           0, b->stats ? b->stats + r : 0,
                           b->node_energy ? b->node_energy + (size_t)r * (size_t)b->N : 0,
                           b->hist ? b->hist + (size_t)r * ORC_HIST_METRICS * ORC_HIST_BINS : 0,
                           b->user ? b->user + r : 0};
        orc_run_rep(&in, &out);
    }
    return 0;
}

int orc_run_batch(int32_t R, int64_t T, int32_t N, int32_t node_stride,
                  const int64_t *arrive_tick, const int32_t *req_mips,
                  const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                  int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                  orc_rep_stats *stats, int threads) {
    return orc_run_batch2(R, T, N, node_stride, ORC_POLICY_REF_V3, arrive_tick, req_mips, mips, dl, ul, init_adv,
                          0, 0, node, status, start_tick, done_tick, stats, 0, 0, threads);
}

int orc_run_batch2(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, int threads) {
    return orc_run_batch3(R, T, N, node_stride, policy, arrive_tick, req_mips, mips, dl, ul, init_adv, p_busy_w,
                          p_idle_w, 0, 0, 0, node, status, start_tick, done_tick, stats, node_energy_j, hist, 0,
                          threads);
}

int orc_run_batch3(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads) {
    return orc_run_batch4(R, T, N, node_stride, policy, arrive_tick, req_mips, mips, dl, ul, init_adv, p_busy_w,
                          p_idle_w, user_ul, user_dl, user_per_task, 0, node, status, start_tick, done_tick, stats,
                          node_energy_j, hist, user_stats, threads);
}

int orc_run_batch4(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads) {
    return orc_run_batch5(R, T, N, node_stride, policy, arrive_tick, req_mips, mips, dl, ul, init_adv, p_busy_w,
                          p_idle_w, user_ul, user_dl, user_per_task, down_tick, 0, 0, 0, node, status, start_tick,
                          done_tick, stats, node_energy_j, hist, user_stats, threads);
}

int orc_run_batch5(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick, const int32_t *region, int32_t hier_threshold_s, int64_t hier_up_tick,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads) {
    return orc_run_batch6(R, T, N, node_stride, policy, arrive_tick, req_mips, mips, dl, ul, init_adv, p_busy_w,
                          p_idle_w, user_ul, user_dl, user_per_task, down_tick, region, hier_threshold_s,
                          hier_up_tick, 0, node, status, start_tick, done_tick, stats, node_energy_j, hist,
                          user_stats, threads);
}

int orc_run_batch6(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick, const int32_t *region, int32_t hier_threshold_s, int64_t hier_up_tick,
                   int32_t flags,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads) {
    batch_t b = {R, N, node_stride, policy, T, arrive_tick, req_mips, mips, dl, ul, init_adv, p_busy_w, p_idle_w,
                 user_ul, user_dl, user_per_task, down_tick, region, hier_threshold_s, hier_up_tick, flags, node,
                 status, start_tick, done_tick, stats, node_energy_j, hist, user_stats, 0};
    pthread_mutex_init(&b.mu, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], 0, batch_worker, &b);
    for (int i = 0; i < threads; i++) pthread_join(th[i], 0);
    pthread_mutex_destroy(&b.mu);
    return ORC_OK;
}
