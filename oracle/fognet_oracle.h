/*
 * fognet_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of FogNetSim++'s offload-decision hot path, written event by
 * event after the reference handlers (BrokerBaseApp3 + ComputeBrokerApp3,
 * OMNeT++ 4.6 sequential kernel semantics).  It is the parity checker for the
 * HIP engine in fognetsimpp_amd/ and the `cpu_baseline` leg of bench.py.
 * Nothing in the product path may link, load or call this code.
 *
 * Parity status: the reference cannot be built or run in this image (it needs
 * OMNeT++ 4.6 + INET 3.3; stand-in headers are not allowed) and it ships no
 * tests and no result files for the v3 modules.  This restatement is therefore
 * pinned only by hand-traced known-answer vectors derived from the reference
 * source (tests/golden/kat_*.json) — formally "parity unpinned" against an
 * executable reference.  See DESIGN.md §2.
 */
#ifndef FOGNET_ORACLE_H
#define FOGNET_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes mirror include/fognet_hip.h */
enum {
    ORC_OK = 0,
    ORC_ERR_ARG = 1,
    ORC_ERR_NO_NODES = 2, /* BrokerBaseApp3.cc:268 reads brokers[0] before the size check (UB) */
    ORC_ERR_DIV0 = 3,     /* BrokerBaseApp3.cc:268 / ComputeBrokerApp3.cc:276 int division by MIPS 0 (SIGFPE) */
    ORC_ERR_STATE = 4,    /* ComputeBrokerApp3.cc:301 scheduleAt() on a pending selfMsg (cRuntimeError) */
    ORC_ERR_OOM = 6,
    ORC_ERR_UNSUPPORTED = 8
};

/* Broker allocation policies (values mirror include/fognet_hip.h). */
enum {
    ORC_POLICY_REF_V3 = 1,  /* BrokerBaseApp3::sendPubAck, BrokerBaseApp3.cc:265-281            */
    ORC_POLICY_EXT_LAT = 16, /* north-star cost (not in the reference): dl_j + busy_j + req/mips_j */
    ORC_POLICY_EXT_HIER = 32 /* hierarchical brokers + mobility handoff (not in the reference; fognet_hip.h) */
};
#define ORC_HIER_REGION_NODES 1024

/* Histograms (fognet_hip.h FOGNET_HIST_*): metric 0 queueTime, 1 response. */
#define ORC_HIST_METRICS 2
#define ORC_HIST_BINS 64

/* One replication: a pre-generated trace replayed through the broker/node handlers. */
typedef struct {
    int32_t n_nodes;
    int64_t n_tasks;
    const int64_t *arrive_tick;   /* [T] publish arrival tick at the broker            */
    const int32_t *req_mips;      /* [T] MqttMsgPublish.MIPSRequired (int)             */
    const int32_t *mips;          /* [N] ComputeBrokerApp3 par("MIPS") (int)           */
    const int64_t *dl_tick;       /* [N] broker -> node delivery latency, ticks        */
    const int64_t *ul_tick;       /* [N] node -> broker delivery latency, ticks        */
    const int64_t *init_adv_tick; /* [N] arrival tick of node's first advertisement    */
    const double *p_busy_w;       /* [N] power while serving, W (nullable: no energy)  */
    const double *p_idle_w;       /* [N] power while idle, W                           */
    int32_t policy;               /* ORC_POLICY_*; 0 means REF_V3                      */
    /* User side (nullable: not modelled).  The publishing user's links: user ->
     * broker (the publish; created = arrive - user_ul) and broker -> user (the
     * pubacks), per task ([T], user_per_task = 1) or one user ([1]). */
    const int64_t *user_ul_tick;
    const int64_t *user_dl_tick;
    int32_t user_per_task;
    /* Node-down extension (not in the reference's scenarios; INET lifecycle,
     * ComputeBrokerApp3::handleNodeCrash, ComputeBrokerApp3.cc:423-427):
     * [N] tick at which node j crashes, INT64_MAX = never; nullable.  The
     * crash precedes every model event of its tick; must be >= init_adv_tick. */
    const int64_t *down_tick;
    /* ORC_POLICY_EXT_HIER: [T] region of each publish's broker, escalation threshold (busy
     * seconds) and the escalated task's extra latency (ticks) */
    const int32_t *region;
    int32_t hier_threshold_s;
    int64_t hier_up_tick;
    /* 1: end the run where the reference ends it, at the first queueTime emission
     * that throws (ComputeBrokerApp3.cc:238; no handler up to :84-86): that
     * RELEASERESOURCE has sent its status-6 ack and lowered busyTime (:228-234)
     * and nothing after the emit runs, no later event either.  Per-task outputs
     * not reached stay -1 (status 0).  0: count the emission and go on (the
     * engine's extension).  Both record abort_tick / abort_task. */
    int32_t stop_at_ref_abort;
} orc_rep_in;

/* Task status of a task that reached a crashed node (no ack, never served). */
#define ORC_TASK_LOST 9

/* count / min / max / exact sum (signed 128-bit) and sum of squares (192-bit,
 * sq_top = bits 128..191) of a signal's raw emitted simtime_t values; overflow
 * counts emissions the reference drops (simtime_t range, orc_ms_raw). */
typedef struct {
    int64_t count, min_raw, max_raw;
    uint64_t sum_lo, sum_hi, sq_lo, sq_hi, sq_top;
    int64_t overflow;
} orc_moments;

/* The user-side signals of the offload loop: broker `delay` (BrokerBaseApp3.cc:143)
 * and mqttApp2's `latency` (status 5, mqttApp2.cc:257-265), `latencyH1`
 * (status 4: the broker's own ack and the node's "queued" relay, :269-277)
 * and `taskTime` (status 6, :279-291). */
typedef struct {
    orc_moments delay, latency, latencyH1, taskTime;
} orc_user_stats;

/* Per-replication statistics (byte layout = fognet_rep_stats, fognet_hip.h).
 * queueTime moments are over the raw simtime_t value the reference emits
 * (orc_qtime_raw), response moments over exact ticks. */
typedef struct {
    int64_t n_tasks, n_queued, n_started;
    int64_t last_tick;
    int64_t queue_min_raw, queue_max_raw, resp_min_ticks, resp_max_ticks;
    /* exact accumulators: queue sum signed two's complement 128-bit, squares 192-bit
     * (queue_sq_top = bits 128..191), response sums unsigned 128-bit */
    uint64_t queue_sum_lo, queue_sum_hi, queue_sq_lo, queue_sq_hi;
    uint64_t resp_sum_lo, resp_sum_hi, resp_sq_lo, resp_sq_hi;
    int64_t events;               /* FES events processed (diagnostic) */
    int32_t max_pending;          /* max tasks assigned-but-not-advertised on one node */
    int32_t status;
    int64_t busy_s;               /* sum of service seconds over all tasks             */
    double energy_j;              /* builder-defined node energy (fognet_hip.h)        */
    uint64_t queue_sq_top;
    int64_t n_qtime;              /* queueTime emissions in the moments                */
    int64_t n_qtime_overflow;     /* emissions at which the reference's simtime_t
                                     arithmetic leaves the int64 range (orc_qtime_raw) */
    int64_t abort_tick;           /* the reference's abort point: tick of the first
                                     overflowing emission (INT64_MAX: none) ...          */
    int64_t abort_task;           /* ... and the task it would have started (-1: none);
                                     at one tick the lowest index (fognet_hip.h)         */
} orc_rep_stats;

/* OMNeT++ 4.6 SimTime at the default scale 1e-12 (include/simtime.h, not in the
 * reference tree; restated): raw int64 t, dbl() = t * 1e-12, SimTime(double d) =
 * toInt64(1e12 * d), SimTime * double = toInt64(t * d), with toInt64(x) =
 * floor(x + 0.5) and a cRuntimeError when that is outside the int64 range.
 *
 * orc_qtime_raw: the raw simtime_t the node emits as queueTime
 * (ComputeBrokerApp3.cc:238) for a task enqueued at tick qstart (queueStartTime
 * = simTime().dbl(), :306, a double) and started at tick now:
 *   (simTime() - SimTime(queueStartTime)) * 1000.
 * Returns 0 when the reference throws there (|...| >= 2^63: a queue time of
 * more than ~9223 s); the recorded value is raw * 1e-12 (dbl()) "ms". */
int orc_qtime_raw(int64_t now, int64_t qstart, int64_t *raw);
/* (simTime() - t0) * 1000 with t0 a simtime_t (mqttApp2.cc:260,272,282): the
 * raw simtime_t of the user-side ms signals; 0 on overflow. */
int orc_ms_raw(int64_t diff_ticks, int64_t *raw);

typedef struct {
    int32_t *node;       /* [T] chosen node index, -1 if never decided (nullable) */
    uint8_t *status;     /* [T] 5 task assigned (idle) / 4 task queued / 9 lost   */
    int64_t *start_tick; /* [T] service start tick (-1: never started)            */
    int64_t *done_tick;  /* [T] RELEASERESOURCE tick (-1: never completed)        */
    double *final_view_busy; /* [N] broker view busyTime after the last event (nullable) */
    orc_rep_stats *stats;
    double *node_energy_j;   /* [N] per-node energy (nullable)                         */
    int64_t *hist;           /* [2][64] histogram counts, ADDED to (nullable)          */
    orc_user_stats *user;    /* user-side signals (needs user_ul/dl_tick; nullable)    */
} orc_rep_out;

int orc_run_rep(const orc_rep_in *in, orc_rep_out *out);

/* Scalar decision core, BrokerBaseApp3.cc:267-281. */
int orc_decide_v3(int32_t n, const double *adv_busy, const int32_t *adv_mips, int32_t req, int32_t *out_node);

/* North-star extension cost (not in the reference): argmin over j of
 * dl_j + adv_busy_j * 1e12 + (req / mips_j) * 1e12 in int64 ticks, ties -> lowest j. */
int orc_decide_ext_lat(int32_t n, const double *adv_busy, const int32_t *mips, const int64_t *dl, int32_t req,
                       int32_t *out_node);

/* Hierarchical brokers (ORC_POLICY_EXT_HIER): the broker of region r takes the
 * smallest (advertised busy, index) among nodes r*1024 .. min(n, r*1024+1024)-1;
 * if that busy exceeds threshold_s the parent takes it over all n nodes
 * (*escalated = 1). */
int orc_decide_hier(int32_t n, const double *adv_busy, const int32_t *adv_mips, int32_t region, int32_t threshold_s,
                    int32_t req, int32_t *out_node, int32_t *escalated);

/* BrokerBaseApp2 (v2 policy) decision, BrokerBaseApp2.cc:180-192 (publish
 * branch) + 235-270 (sendPubAck(status=false)): served by the broker itself if
 * MIPSRequired < its own MIPS; otherwise the node is the LAST index i >= 1
 * whose advertised MIPS exceeds node 0's (temp is never updated, :241-248),
 * else 0, and the task is sent only if MIPSRequired < that node's MIPS.
 * *out_action: ORC_V2_* below; *out_node: the chosen node (-1 for LOCAL and
 * NO_NODES). */
enum {
    ORC_V2_LOCAL = 3,    /* pubAck status 3, the broker reserves its own MIPS (:181-182, :209-232) */
    ORC_V2_FORWARD = 4,  /* pubAck status 4 + FognetMsgTask to the node (:186-192, :262-270)        */
    ORC_V2_DROPPED = 5,  /* pubAck status 4 but MIPSRequired >= the node's MIPS: no task (:262)      */
    ORC_V2_NO_NODES = 6  /* "no compute resource available" (:273-285)                             */
};
int orc_decide_v2(int32_t n, const int32_t *adv_mips, int32_t local_mips, int32_t req, int32_t *out_node,
                  int32_t *out_action);

/* ---- v2 model replay (fognet_oracle_v2.c): BrokerBaseApp2 + ComputeBrokerApp2 */

/* per-task outcome */
enum {
    ORC_V2_ST_LOCAL = 3,      /* reserved in the broker's own pool (pubAck 3)                  */
    ORC_V2_ST_FORWARDED = 4,  /* FognetMsgTask sent, not yet at the node when the run stopped  */
    ORC_V2_ST_DROPPED = 5,    /* pubAck 4 but MIPSRequired >= the chosen node's advertised MIPS */
    ORC_V2_ST_NO_NODES = 6,   /* no compute broker registered                                  */
    ORC_V2_ST_ACCEPTED = 7,   /* reserved at the node (TaskAck true, ComputeBrokerApp2.cc:269)  */
    ORC_V2_ST_REJECTED = 8    /* MIPSRequired >= the node's remaining MIPS (TaskAck false)      */
};

typedef struct {
    int32_t n_nodes;
    int64_t n_tasks;
    const int64_t *arrive_tick;    /* [T] publish arrival at the broker, nondecreasing          */
    const int32_t *req_mips;       /* [T] MqttMsgPublish.MIPSRequired                            */
    double required_time;          /* MqttMsgPublish.requiredTime, s (mqttApp2.cc:372: 0.01)     */
    int32_t broker_mips;           /* BrokerBaseApp2 par("MIPS") (wirelessNet.ini:58)            */
    const int32_t *mips;           /* [N] ComputeBrokerApp2 par("MIPS") (wirelessNet.ini:64)     */
    const int64_t *dl_tick;        /* [N] broker -> node latency                                 */
    const int64_t *ul_tick;        /* [N] node -> broker latency                                 */
    const int64_t *first_adv_tick; /* [N] first ADVERTISEMIPS firing at the node                 */
    int64_t stop_tick;             /* sim-time-limit: events at ticks >= stop are not processed  */
} orc_v2_in;

typedef struct {
    int64_t n_tasks, n_local, n_forwarded, n_accepted, n_rejected, n_dropped, n_no_nodes;
    int64_t n_released_broker;  /* broker RELEASERESOURCE releases (BrokerBaseApp2.cc:382-406)     */
    int64_t n_inflated;         /* ... of them forwarded requests credited to the broker's pool    */
    int64_t n_released_node;    /* node releases (ComputeBrokerApp2.cc:222-245)                   */
    int64_t n_relayed;          /* status-6 acks that found their request at the broker (:143-154) */
    int64_t events;             /* events processed (cancelled timers excluded)                    */
    int64_t node_mips_final_sum;
    int32_t broker_mips_final;
    int32_t status;
} orc_v2_stats;

typedef struct {
    int32_t *node;        /* [T] chosen node, -1: served locally / no node (nullable)   */
    uint8_t *status;      /* [T] ORC_V2_ST_* (0: not published before the stop)         */
    int64_t *start_tick;  /* [T] reservation tick, -1 if never reserved                 */
    int64_t *done_tick;   /* [T] release tick of its reservation, -1 if not released    */
    orc_v2_stats *stats;
} orc_v2_out;

int orc_run_v2_rep(const orc_v2_in *in, orc_v2_out *out);

typedef struct {
    int32_t R, N, node_stride;
    int64_t T;
    const int64_t *arrive_tick; const int32_t *req_mips;            /* [R][T] */
    const double *required_time; const int32_t *broker_mips;        /* [R]    */
    const int64_t *stop_tick;                                       /* [R]    */
    const int32_t *mips; const int64_t *dl_tick, *ul_tick, *first_adv_tick; /* [R|1][N] */
    int32_t *node; uint8_t *status; int64_t *start_tick, *done_tick; /* [R][T] (nullable) */
    orc_v2_stats *stats;                                            /* [R]    */
} orc_v2_batch;
int orc_run_v2_batch(const orc_v2_batch *b, int threads);

/* Histogram bin of a duration in ticks (fognet_hip.h FOGNET_HIST_BINS rule) and of a
 * raw emitted ms signal (bin of the recorded double raw * 1e-12 ms). */
int orc_hist_bin(int64_t ticks);
int orc_hist_bin_raw(int64_t raw);

/* Batch of R replications sharing T and N; node params have stride node_stride
 * (0 = shared).  Runs on `threads` pthreads, one replication per thread at a time. */
int orc_run_batch(int32_t R, int64_t T, int32_t N, int32_t node_stride,
                  const int64_t *arrive_tick, const int32_t *req_mips,
                  const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                  int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                  orc_rep_stats *stats, int threads);

/* The same with a policy, an optional power model ([R|1][N], node_stride) and
 * optional per-node energy [R][N] and per-replication histograms [R][2][64]. */
/* orc_run_batch2 + the user side: user_ul/user_dl [R][T] (user_per_task) or
 * [R] (one user per replication); user_stats [R] (nullable). */
int orc_run_batch3(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads);

/* orc_run_batch3 plus the node-down extension: down_tick [R|1][N] (nullable). */
/* orc_run_batch4 + the EXT_HIER inputs: region [R][T] (nullable), threshold, up latency. */
int orc_run_batch5(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick, const int32_t *region, int32_t hier_threshold_s, int64_t hier_up_tick,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads);

/* orc_run_batch5 + flags (bit 0: orc_rep_in.stop_at_ref_abort). */
int orc_run_batch6(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick, const int32_t *region, int32_t hier_threshold_s, int64_t hier_up_tick,
                   int32_t flags,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads);

int orc_run_batch4(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   const int64_t *user_ul, const int64_t *user_dl, int32_t user_per_task,
                   const int64_t *down_tick,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, orc_user_stats *user_stats,
                   int threads);

int orc_run_batch2(int32_t R, int64_t T, int32_t N, int32_t node_stride, int32_t policy,
                   const int64_t *arrive_tick, const int32_t *req_mips,
                   const int32_t *mips, const int64_t *dl, const int64_t *ul, const int64_t *init_adv,
                   const double *p_busy_w, const double *p_idle_w,
                   int32_t *node, uint8_t *status, int64_t *start_tick, int64_t *done_tick,
                   orc_rep_stats *stats, double *node_energy_j, int64_t *hist, int threads);

#ifdef __cplusplus
}
#endif
#endif
