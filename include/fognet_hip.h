/*
 * fognet_hip.h — C ABI of libfognet_hip, the MI355X (gfx950) engine for
 * FogNetSim++'s offload-decision hot path.
 *
 * Reference interfaces replaced (paths relative to the FogNetSim++ tree):
 *   - the broker's allocation argmin, BrokerBaseApp3::sendPubAck(status=false),
 *     src/mqttapp/BrokerBaseApp3.cc:265-304 (decision core :267-281)
 *       -> fognet_decide / fognet_decide_batch_dev;
 *   - the v2 broker's local-first / "max-MIPS" forward, BrokerBaseApp2.cc:180-192
 *     and :235-286 -> fognet_decide_v2 / fognet_decide_v2_batch_dev;
 *   - the fog node's task arrival, ComputeBrokerApp3::processPacket,
 *     src/mqttapp/ComputeBrokerApp3.cc:269-320, its completion + advertisement,
 *     ComputeBrokerApp3::releaseResource / advertiseMIPS, :224-256 / :205-222,
 *     and the broker's view update on each advertisement,
 *     BrokerBaseApp3.cc:123-130 -> fognet_run_batch[_dev] (R independent
 *     trace replays of the whole decide -> queue -> complete -> advertise loop);
 *   - the queueTime statistic (ComputeBrokerApp3.cc:238, ComputeBrokerApp3.ned:45-46)
 *     -> fognet_rep_stats, reduced on the device (fognet_reduce_stats_dev);
 *   - the ack relay and the users' latency signals (BrokerBaseApp3.cc:143,
 *     164-198; mqttApp2.cc:252-291) -> fognet_user_stats_dev.
 *
 * Conventions
 *   - Every entry point returns a fognet_status; no exception crosses the ABI.
 *     fognet_last_error() gives the message of the last failure on a context.
 *   - The caller owns every buffer.  *_dev entry points take device pointers
 *     (hipMalloc'd, or torch.cuda tensors) and enqueue on the given hipStream_t
 *     (NULL = default stream); the others take host pointers and copy.
 *   - A fognet_ctx is not thread-safe; use one per host thread (OMNeT++'s
 *     sequential kernel is single-threaded anyway).
 *   - Deterministic: identical inputs give bit-identical outputs.
 *   - Time is OMNeT++ 4.6 simtime_t raw int64 at scale 1e-12 s ("ticks").
 */
#ifndef FOGNET_HIP_H
#define FOGNET_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FOGNET_ABI_VERSION 10
#define FOGNET_TICKS_PER_SECOND 1000000000000LL

/* Latency histograms (device-side statistics, summed over replications; the
 * only data the multi-GPU path all-reduces over RCCL together with energy).
 * Metric 0 = queueTime (ComputeBrokerApp3.cc:238, queued tasks only): q = the
 * whole part of the recorded value in ms (the emitted raw simtime_t * 1e-12,
 * see "Reference signal values" below); metric 1 = response (completion tick -
 * publish tick at the broker): q = ticks / 10^9 whole milliseconds.  A value
 * falls in bin 0 if q < 1, else min(63, floor(log2 q) + 1): bin b >= 1 holds
 * [2^(b-1), 2^b) ms. */
#define FOGNET_HIST_METRICS 2
#define FOGNET_HIST_BINS 64

typedef int64_t fognet_tick;
typedef struct fognet_ctx fognet_ctx;

typedef enum fognet_status {
    FOGNET_OK = 0,
    FOGNET_ERR_ARG = 1,         /* invalid argument / precondition (see fognet_run_batch)            */
    FOGNET_ERR_NO_NODES = 2,    /* n == 0: BrokerBaseApp3.cc:268 reads brokers[0] first (UB)           */
    FOGNET_ERR_DIV0 = 3,        /* advertised MIPS of node 0 is 0: BrokerBaseApp3.cc:268 SIGFPE        */
    FOGNET_ERR_STATE = 4,       /* scheduleAt on a scheduled selfMsg (ComputeBrokerApp3.cc:301): the
                                   reference's cRuntimeError is swallowed by processPacket's catch
                                   (:277,317), leaving the node busy with no completion pending;
                                   unreachable under the fognet_batch_in preconditions            */
    FOGNET_ERR_DEVICE = 5,      /* HIP runtime failure or no gfx950 device                             */
    FOGNET_ERR_OOM = 6,
    FOGNET_ERR_CAPACITY = 7,    /* v2 queue_capacity exceeded; a decision whose smallest advertised busy
                                   time is 2^32 - 1 s or more (the view keeps 32 bits, saturated: larger
                                   values only lose); EXT_LAT: an advertised busy time of 2^24 s or more */
    FOGNET_ERR_UNSUPPORTED = 8, /* configuration not implemented (e.g. N > 2^20, unknown policy)     */
    FOGNET_REF_ABORTED = 9,     /* replication status under FOGNET_FLAG_REF_ABORT: the reference run ends
                                   at a queueTime emission that overflows (ComputeBrokerApp3.cc:238; see
                                   "Reference signal values"); outputs are still written in full     */
    FOGNET_ERR_INTERNAL = 10    /* an internal invariant check of the replay failed (a library bug)   */
} fognet_status;

/* fognet_batch_in.flags */
#define FOGNET_FLAG_REF_ABORT 1 /* a replication the reference would abort (abort_tick set) gets status
                                   FOGNET_REF_ABORTED, so job reductions count it as failed, as the
                                   reference records no result for it; without the flag its status is
                                   FOGNET_OK and the continuation past the abort is the extension's */

typedef enum fognet_policy {
    FOGNET_POLICY_REF_V2 = 2,   /* BrokerBaseApp2: local-first, then the LAST node whose advertised MIPS
                                   exceeds node 0's, forwarded only if MIPSRequired < its MIPS
                                   (fognet_decide_v2; needs the broker's own MIPS)                 */
    FOGNET_POLICY_REF_V3 = 1,   /* BrokerBaseApp3: argmin(busy_j + req / mips_0), int division,
                                   strict '<' (ties -> lowest index), stale advertised view      */
    FOGNET_POLICY_EXT_LAT = 16, /* north-star cost, NOT in the reference (parity vs the oracle's
                                   restatement only): argmin over j of
                                   dl_j + adv_busy_j * 1e12 + (req / mips_j) * 1e12 ticks
                                   (int division by the node's OWN MIPS, exact int64 ticks,
                                   ties -> lowest index); same stale view and node model      */
    FOGNET_POLICY_EXT_HIER = 32 /* hierarchical brokers with mobility handoff (BASELINE.json C5), NOT
                                   in the reference (one flat broker, BrokerBaseApp3.cc:271-279):
                                   the nodes form regions of FOGNET_HIER_REGION_NODES consecutive
                                   indices, each with a regional broker; publish t reaches the
                                   broker of region[t] (the user's region when it publishes: a
                                   handoff changes it).  That broker applies BrokerBaseApp3's rule
                                   inside its region: the smallest (advertised busy, index).  If
                                   that busy exceeds hier_threshold_s the task is escalated to the
                                   parent broker, which applies the rule over ALL nodes, and
                                   reaches its node hier_up_tick later (the extra hop).  Adverts
                                   reach every broker with the node's uplink latency.  A direct
                                   task can reach a node before an escalated task decided earlier
                                   (it overtakes it inside the hop): the node serves in arrival
                                   order; any number of escalated tasks may be in flight at once
                                   (the node FIFO takes any length, ComputeBrokerApp3.cc:305-309).
                                   A replication that fails (status != OK) leaves the per-task
                                   outputs of escalated tasks still in flight at the error
                                   unwritten, like every task after the error.                */
} fognet_policy;

/* Region size of FOGNET_POLICY_EXT_HIER (node r * 1024 .. r * 1024 + 1023 form region r). */
#define FOGNET_HIER_REGION_NODES 1024

/* Outcome of one BrokerBaseApp2 decision (BrokerBaseApp2.cc:180-192, 235-286). */
typedef enum fognet_v2_action {
    FOGNET_V2_LOCAL = 3,     /* MIPSRequired < the broker's own MIPS: served locally (pubAck status 3)  */
    FOGNET_V2_FORWARD = 4,   /* pubAck status 4 + FognetMsgTask to *out_node                            */
    FOGNET_V2_DROPPED = 5,   /* pubAck status 4, MIPSRequired >= the chosen node's MIPS: no task sent   */
    FOGNET_V2_NO_NODES = 6   /* no compute broker registered: "no compute resource available" puback   */
} fognet_v2_action;

/* Reference signal values.  The reference emits its latency signals as
 * simtime_t values (OMNeT++ 4.6, scale 1e-12: a raw int64 t, recorded as the
 * double dbl() = t * 1e-12), and computes them with SimTime's double round
 * trips: SimTime(double d) = toInt64(1e12 * d), SimTime * double =
 * toInt64(t * d), toInt64(x) = floor(x + 0.5), a cRuntimeError outside int64.
 * The statistics keep exact moments of those RAW emitted values ("raw"):
 *   queueTime  (simTime() - SimTime(queueStartTime)) * 1000, queueStartTime =
 *              simTime().dbl() of the enqueue, a double (ComputeBrokerApp3.cc:238,
 *              306, Request.cc:26): raw = toInt64((double)(now -
 *              toInt64(1e12 * (a * 1e-12))) * 1000.0) for a task enqueued at tick a
 *              and started at tick now (the recorded value, raw * 1e-12, is in ms;
 *              it can be a few ulps off the exact tick difference, even negative
 *              for a task queued and started in the same tick);
 *   latency / latencyH1 / taskTime  (simTime() - timeCreated) * 1000 with
 *              timeCreated a simtime_t (mqttApp2.cc:260,272,282): raw = toInt64(d * 1000.0);
 *   delay      simTime() - creationTime (BrokerBaseApp3.cc:143): raw = d ticks (s).
 * An emission whose product leaves the int64 range (a queue time above ~9223 s)
 * throws in the reference.  At the user signals the exception is swallowed by
 * mqttApp2's catch and the emission is lost (fognet_moments.overflow).  At
 * queueTime it ENDS THE REFERENCE RUN: ComputeBrokerApp3::releaseResource emits
 * at ComputeBrokerApp3.cc:238 before it dequeues the next task (:240-250) and
 * nothing up to handleMessageWhenUp (:84-86) catches, so OMNeT++ stops at that
 * RELEASERESOURCE event.  The engine reports that point per replication
 * (fognet_rep_stats.abort_tick / abort_task) and, as a builder-defined
 * EXTENSION of the reference, keeps replaying past it: the emission is counted
 * (n_qtime_overflow) and left out of the moments and histograms, and the node
 * dequeues its next task as if the emit had returned.  What the reference
 * defines of an aborted replication is the prefix before that event: every
 * publish with arrive_tick <= abort_tick is decided (trace publishes precede
 * same-tick dynamic events), and every arrival, start and
 * completion at a tick < abort_tick has happened.  Everything later, and every
 * statistic that includes it, is the extension's.  Signed sums are two's
 * complement. */

/* Per-replication statistics.  Exact integer moments, split into uint64 limbs
 * ([lo, hi, top] = bits 0-63, 64-127, 128-191) so results are bit-reproducible. */
typedef struct fognet_rep_stats {
    int64_t n_tasks;          /* decisions made                                                   */
    int64_t n_queued;         /* node acks with status 4 ("task queued", :310-313)                 */
    int64_t n_started;        /* node acks with status 5                                          */
    int64_t last_tick;        /* latest RELEASERESOURCE tick (makespan)                           */
    int64_t queue_min_raw, queue_max_raw;     /* queueTime emissions: raw values (see above)       */
    int64_t resp_min_ticks, resp_max_ticks;   /* over all tasks: done - arrival at broker          */
    uint64_t queue_sum_lo, queue_sum_hi;      /* signed 128-bit sum of queueTime raw values        */
    uint64_t queue_sq_lo, queue_sq_hi;        /* bits 0-127 of the sum of their squares            */
    uint64_t resp_sum_lo, resp_sum_hi, resp_sq_lo, resp_sq_hi;
    int64_t events;           /* reference FES events this replay stands for (2N + 4 per task)    */
    int32_t max_pending;      /* max tasks assigned to one node whose completion advert had not
                                 reached the broker yet (ring occupancy)                          */
    int32_t status;           /* fognet_status of this replication                                */
    int64_t busy_s;           /* sum of service seconds (req / MIPS) over all tasks               */
    double energy_j;          /* node energy (builder-defined, not in the reference; 0 when no
                                 power model): sum over j in index order of
                                 P_busy_j * B_j + P_idle_j * ((H - B_j * 1e12) / 1e12), with
                                 B_j = node j's service seconds, H = last_tick (0 if no task);
                                 IEEE fp64, no fused multiply-add                                 */
    uint64_t queue_sq_top;    /* bits 128-191 of the queueTime sum of squares                     */
    int64_t n_qtime;          /* queueTime emissions in the moments (queued tasks that started)   */
    int64_t n_qtime_overflow; /* queueTime emissions the reference cannot make (simtime overflow) */
    /* The reference's abort point (see "Reference signal values"): the RELEASERESOURCE
     * tick at which the first overflowing queueTime emission throws and the index of the
     * task it would have started; INT64_MAX / -1 when the reference run completes.
     * Several overflowing emissions at that tick (different nodes): the lowest task index
     * (the reference throws at the first in FES insertion order, which this does not
     * resolve; the tick and so the reference-defined prefix are the same). */
    int64_t abort_tick;
    int64_t abort_task;
} fognet_rep_stats;

/* Job-level statistics: the exact sum of any set of fognet_rep_stats.  Sums
 * are 192-bit integers (limbs [0] = least significant; queue_sum two's
 * complement), so combining is associative and the integer fields do not
 * depend on how replications were sharded over GPUs.  Mean/stddev in ms:
 * queueTime sum * 1e-12 / n_qtime, response sum / n_tasks / 1e9, etc. */
typedef struct fognet_job_stats {
    int64_t n_reps, n_failed;
    int64_t n_tasks, n_queued, n_started;
    int64_t last_tick;
    int64_t queue_min_raw, queue_max_raw, resp_min_ticks, resp_max_ticks;
    uint64_t queue_sum[3], queue_sq[3], resp_sum[3], resp_sq[3];
    int64_t events;
    int64_t max_pending;
    int64_t busy_s;
    double energy_j;          /* fp64 sum over replications: fixed tree order on one device, rank
                                 order across GPUs; differs from another sharding's sum by
                                 rounding only (within 1e-9 relative)                            */
    int64_t n_qtime, n_qtime_overflow;
    int64_t n_ref_aborted;    /* replications the reference would have aborted (abort_tick set),
                                 status OK or FOGNET_REF_ABORTED (the latter also in n_failed) */
} fognet_job_stats;

/* R trace replays of T tasks over N fog nodes, SoA, row-major [R][T] / [R|1][N]. */
typedef struct fognet_batch_in {
    int32_t R, T, N;
    int32_t policy;           /* fognet_policy                                                    */
    int32_t node_stride;      /* 0: node params shared by all replications; N: one row each       */
    int32_t ring_capacity;    /* per-node pending-task ring of the register-resident replay kernel
                                 (N <= 256), power of two in [2, 2^15] (0 = default 2048).  Not a
                                 limit on the inputs: a replication with a node past it (or with a
                                 service time past min(2^24 / ring_capacity, 255) s, or a task
                                 reaching its node past 2^56 ticks, the 8-B ring entry's ranges) is
                                 replayed again from the start by the wide kernel, whose per-node
                                 chains are unbounded, inside the same call.  Only sizes the
                                 workspace (8 B per entry) and the common path.                  */
    const int64_t *arrive_tick;   /* [R][T] publish arrival at the broker, nondecreasing          */
    const int32_t *req_mips;      /* [R][T] MqttMsgPublish.MIPSRequired, >= 0                      */
    const int32_t *mips;          /* [R|1][N] node MIPS (> 0), CONNECT order = index order         */
    const int64_t *dl_tick;       /* [R|1][N] broker -> node delivery latency (>= 0)               */
    const int64_t *ul_tick;       /* [R|1][N] node -> broker delivery latency (>= 0)               */
    const int64_t *init_adv_tick; /* [R|1][N] arrival of the node's first advert at the broker;
                                     ul <= init_adv < arrive[0] (all adverts land before task 0)  */
    const double *p_busy_w;       /* [R|1][N] node power while serving, W (nullable: no energy)   */
    const double *p_idle_w;       /* [R|1][N] node power while idle, W (null iff p_busy_w is)     */
    /* Node-down extension (not one of the reference's scenarios): [R|1][N] tick at which
     * node j crashes (INT64_MAX = never; otherwise init_adv_tick <= down < 2^61), nullable.
     * INET lifecycle, ComputeBrokerApp3::handleNodeCrash (ComputeBrokerApp3.cc:423-427):
     * the node's RELEASERESOURCE timer is cancelled and the host drops arriving tasks;
     * the broker keeps its last advert.  The crash precedes every model event of its
     * tick.  Replays with crashes run on the wide kernel; not combinable with the power
     * model (ERR_UNSUPPORTED); not stored in trace files (fognet_io.h). */
    const int64_t *down_tick;
    /* FOGNET_POLICY_EXT_HIER only (ignored otherwise): [R][T] region of each publish's
     * regional broker (0 <= region < ceil(N / FOGNET_HIER_REGION_NODES)), the busy seconds
     * above which a regional broker escalates, the extra latency of an escalated task. */
    const int32_t *region;
    int64_t hier_up_tick;
    int32_t hier_threshold_s;
    int32_t flags;            /* FOGNET_FLAG_* (0: none)                                           */
} fognet_batch_in;

/* Per-task status (fognet_batch_out.status). */
typedef enum fognet_task_status {
    FOGNET_TASK_QUEUED = 4,   /* node ack "task queued"   (ComputeBrokerApp3.cc:304-313)       */
    FOGNET_TASK_STARTED = 5,  /* node ack "task assigned" (ComputeBrokerApp3.cc:282-301)       */
    FOGNET_TASK_LOST = 9      /* reached a crashed node (down_tick): no ack, never served       */
} fognet_task_status;

typedef struct fognet_batch_out {
    int32_t *node;            /* [R][T] chosen node                                               */
    uint8_t *status;          /* [R][T] fognet_task_status: 5 started on arrival, 4 queued, 9 lost */
    int64_t *start_tick;      /* [R][T] service start (-1: never started, node-down only)         */
    int64_t *done_tick;       /* [R][T] completion (RELEASERESOURCE) tick (-1: never, node-down)  */
    fognet_rep_stats *stats;  /* [R], required.  node/status/start_tick/done_tick: all four, or all
                                 NULL for a statistics-only replay (fognet_run_batch_dev /
                                 fognet_run_batch only): the caller gets the records and the
                                 histogram; N > 256 (wide kernel) then writes nothing per task,
                                 N <= 256 keeps the per-task outputs in the context's workspace
                                 for its fused statistics pass                                 */
    double *node_energy_j;    /* [R][N] per-node energy (nullable; needs the power model)         */
    int64_t *hist;            /* [FOGNET_HIST_METRICS][FOGNET_HIST_BINS] job histogram, ADDED to
                                 (the caller zeroes it; nullable)                                 */
} fognet_batch_out;

/* count / min / max / exact signed 128-bit sum and 192-bit sum of squares of a
 * signal's raw emitted values (min_raw = INT64_MAX, max_raw = INT64_MIN when
 * count == 0); overflow: emissions lost to the simtime_t range (see above). */
typedef struct fognet_moments {
    int64_t count, min_raw, max_raw;
    uint64_t sum_lo, sum_hi, sq_lo, sq_hi, sq_top;
    int64_t overflow;
} fognet_moments;

/* User-side signals of one replication, as raw emitted
 * values (see "Reference signal values"): delay in ticks (s), the others the
 * raw simtime_t of (simTime() - created) * 1000 (recorded value raw * 1e-12 ms):
 *   delay      broker `delay` (BrokerBaseApp3.cc:143): publish arrival at the
 *              broker - creation at the user, every publish
 *   latency    mqttApp2 on the relayed status-5 ack ("task assigned",
 *              mqttApp2.cc:257-265)
 *   latencyH1  on status-4 acks (mqttApp2.cc:269-277): the broker's own pubAck
 *              (BrokerBaseApp3.cc:145-150) for every publish, plus the node's
 *              relayed "task queued" ack
 *   taskTime   on the relayed status-6 ack ("performed", mqttApp2.cc:279-291)
 * Acks travel node -> broker (ul_k), are relayed to the request's user
 * (BrokerBaseApp3.cc:164-198) and arrive one user downlink later.  Message
 * ids are assumed unique (the reference matches them with strcmp). */
typedef struct fognet_user_stats {
    fognet_moments delay, latency, latencyH1, taskTime;
} fognet_user_stats;

/* ---- v2 model replay: BrokerBaseApp2 + ComputeBrokerApp2,
 * the modules simulations/example/wirelessNet.ini:56,62 select.  The broker
 * keeps its own MIPS pool with a single RELEASERESOURCE timer
 * (BrokerBaseApp2.cc:205-233, 382-406) and forwards to the LAST node whose
 * advertised MIPS exceeds node 0's (:235-271); a node reserves MIPS for
 * requiredTime and runs a 10-ms advert/release timer (ComputeBrokerApp2.cc:
 * 202-318).  Deadlines are doubles compared with simTime().dbl() = ticks *
 * 1e-12, exactly as the reference does (their rounding decides releases). */
#define FOGNET_V2_MAX_NODES 16384 /* node j on lane j % 64, slot j / 64 (up to 256 per lane) */
/* Device workspace of a v2 replay (fognet_run_v2_dev, allocated and kept by the context): 64 B per
 * (replication, node slot, queue entry) plus R * T B, i.e. R * S * queue_capacity * 64 B with S = N
 * rounded up to 64 x a power of two -- at N = 4096 and the default capacity 256, 64 MiB per replication
 * (128 MiB at N = 8192, 256 MiB at N = 16384).  Above 256 nodes (NPL >= 8) each node's record lives in
 * per-lane scratch memory. */

typedef enum fognet_v2_task_status {
    FOGNET_V2_ST_LOCAL = 3,      /* reserved in the broker's own pool (pubAck 3)                   */
    FOGNET_V2_ST_FORWARDED = 4,  /* task sent, still in flight when the run stopped                */
    FOGNET_V2_ST_DROPPED = 5,    /* MIPSRequired >= the chosen node's advertised MIPS: no task sent */
    FOGNET_V2_ST_NO_NODES = 6,   /* no compute broker registered                                   */
    FOGNET_V2_ST_ACCEPTED = 7,   /* reserved at the node (ComputeBrokerApp2.cc:269-295)             */
    FOGNET_V2_ST_REJECTED = 8    /* MIPSRequired >= the node's remaining MIPS (:299-306)            */
} fognet_v2_task_status;

typedef struct fognet_v2_in {
    int32_t R, T, N;              /* N <= FOGNET_V2_MAX_NODES                                      */
    int32_t node_stride;          /* 0: node parameters shared; N: one row per replication         */
    int32_t queue_capacity;       /* per-node capacity of each message queue and of the
                                     reservation list, power of two (0 = default 256)              */
    int32_t pad;
    const int64_t *arrive_tick;   /* [R][T] publish arrival at the broker, nondecreasing           */
    const int32_t *req_mips;      /* [R][T] MIPSRequired                                           */
    const int32_t *broker_mips;   /* [R] BrokerBaseApp2 par("MIPS")                                */
    const double *required_time_s;/* [R] MqttMsgPublish.requiredTime (mqttApp2.cc:372: 0.01)      */
    const int64_t *stop_tick;     /* [R] sim-time-limit: events at >= stop are not run (<= 2^53)   */
    const int32_t *mips;          /* [R|1][N] ComputeBrokerApp2 par("MIPS")                        */
    const int64_t *dl_tick;       /* [R|1][N] broker -> node latency                               */
    const int64_t *ul_tick;       /* [R|1][N] node -> broker latency                               */
    const int64_t *first_adv_tick;/* [R|1][N] first ADVERTISEMIPS firing (CONNACK + 0.01 s)        */
} fognet_v2_in;

typedef struct fognet_v2_stats {
    int64_t n_tasks, n_local, n_forwarded, n_accepted, n_rejected, n_dropped, n_no_nodes;
    int64_t n_released_broker;    /* broker timer releases (BrokerBaseApp2.cc:382-406)            */
    int64_t n_inflated;           /* ... of forwarded requests, credited to the broker's own pool  */
    int64_t n_released_node;      /* node releases (ComputeBrokerApp2.cc:222-245)                 */
    int64_t n_relayed;            /* status-6 acks that found their request at the broker         */
    int64_t events;               /* events processed (cancelled timers excluded)                  */
    int64_t node_mips_final_sum;
    int32_t broker_mips_final;
    int32_t status;               /* fognet_status of the replication                              */
} fognet_v2_stats;

typedef struct fognet_v2_out {
    int32_t *node;                /* [R][T] chosen node, -1: served locally / no node              */
    uint8_t *status;              /* [R][T] fognet_v2_task_status (0: not published before stop)  */
    int64_t *start_tick;          /* [R][T] reservation tick, -1 if never reserved                 */
    int64_t *done_tick;           /* [R][T] release tick of the reservation, -1 if not released    */
    fognet_v2_stats *stats;       /* [R]                                                           */
} fognet_v2_out;

/* R v2 replays on the device (device pointers; enqueued on hip_stream). */
int fognet_run_v2_dev(fognet_ctx *ctx, const fognet_v2_in *in, fognet_v2_out *out, void *hip_stream);

/* Synthetic trace recipe, generated on the device.
 * Replication r uses Philox4x32-10 key (seed, r); see DESIGN.md §Trace generator. */
typedef struct fognet_gen_params {
    uint32_t seed;
    int32_t req_lo, req_hi;       /* req ~ U_int[req_lo, req_hi]                                  */
    int32_t pad;
    const double *mean_gap_ticks; /* [R] exponential inter-arrival mean per replication (device)  */
    const int64_t *lat_scale;     /* [R] latency multiplier per replication (device)              */
} fognet_gen_params;

int fognet_abi_version(void);
const char *fognet_status_string(int status);

/* Context: binds a HIP device (gfx950 required), owns the replay workspace. */
int fognet_create(fognet_ctx **out, int hip_device);
void fognet_destroy(fognet_ctx *ctx);
const char *fognet_last_error(const fognet_ctx *ctx);

/* Scalar drop-in for BrokerBaseApp3.cc:267-281 (the OMNeT++ adapter's call,
 * INTEGRATION.md §1): host arrays of the broker's advertised view
 * (Broker::busyTime, Broker::MIPS in CONNECT order); evaluated on the device
 * with the reference's exact fp64 arithmetic.  policy: FOGNET_POLICY_REF_V3.
 * One kernel launch per call (views of <= 256 nodes travel in the kernel
 * arguments, larger ones in one DMA copy; the result is written to mapped
 * host memory) and one stream synchronisation. */
int fognet_decide(fognet_ctx *ctx, int policy, int32_t n, const double *adv_busy,
                  const int32_t *adv_mips, int32_t req_mips, int32_t *out_node);

/* The publishes of one window decided together: m requests against ONE view
 * (the broker's view only changes when an advert arrives, BrokerBaseApp3.cc:
 * 123-130, so every publish between two adverts sees the same view).  Equals
 * m fognet_decide calls on that view; one launch, one synchronisation.
 * out_node [m] (host).  Returns the first failing request's status. */
int fognet_decide_window(fognet_ctx *ctx, int policy, int32_t n, const double *adv_busy,
                         const int32_t *adv_mips, int32_t m, const int32_t *req_mips, int32_t *out_node);

/* M independent decisions, device pointers: adv_busy/adv_mips [M][n], req [M],
 * out_node [M], out_status [M] (fognet_status per query, nullable). */
int fognet_decide_batch_dev(fognet_ctx *ctx, int policy, int64_t m, int32_t n,
                            const double *adv_busy, const int32_t *adv_mips, const int32_t *req,
                            int32_t *out_node, int32_t *out_status, void *hip_stream);

/* Drop-in for the v2 broker's allocation (BrokerBaseApp2.cc:180-192 and
 * sendPubAck(status=false) :235-286): host arrays of the advertised MIPS view
 * adv_mips[n] (Broker::MIPS, updated by adverts :128-136), the broker's own
 * remaining MIPS (par MIPS minus local reservations) and MIPSRequired.
 * *out_action: fognet_v2_action; *out_node: chosen node, -1 for LOCAL/NO_NODES.
 * Evaluated on the device. */
int fognet_decide_v2(fognet_ctx *ctx, int32_t n, const int32_t *adv_mips, int32_t local_mips,
                     int32_t req_mips, int32_t *out_node, int32_t *out_action);

/* M independent v2 decisions, device pointers: adv_mips [M][n], local_mips [M],
 * req [M], out_node [M], out_action [M]. */
int fognet_decide_v2_batch_dev(fognet_ctx *ctx, int64_t m, int32_t n, const int32_t *adv_mips,
                               const int32_t *local_mips, const int32_t *req, int32_t *out_node,
                               int32_t *out_action, void *hip_stream);

/* Batched replay engine.  *_dev: every pointer in in/out is a device pointer
 * (the structs themselves are host memory).  Returns FOGNET_OK once enqueued;
 * per-replication failures are reported in stats[r].status. */
int fognet_run_batch_dev(fognet_ctx *ctx, const fognet_batch_in *in, fognet_batch_out *out,
                         void *hip_stream);
/* The two stages fognet_run_batch_dev enqueues, exposed so callers can time or
 * overlap them: the replay kernel (decisions, node queues, adverts; fills
 * node/status/start/done and stats[r].{status,n_tasks,max_pending,events}) and
 * the statistics pass over its outputs (the remaining stats fields). */
int fognet_replay_dev(fognet_ctx *ctx, const fognet_batch_in *in, fognet_batch_out *out, void *hip_stream);
int fognet_rep_stats_dev(fognet_ctx *ctx, const fognet_batch_in *in, fognet_batch_out *out, void *hip_stream);
/* Host-buffer variant: copies in, replays, copies out, synchronises.  Returns
 * the first non-OK replication status, if any. */
int fognet_run_batch(fognet_ctx *ctx, const fognet_batch_in *in, fognet_batch_out *out);

/* User-side signals from a finished replay (fognet_replay_dev or
 * fognet_run_batch_dev on the same stream): device pointers in `in` (trace,
 * node parameters) and `out` (node, status, done_tick, stats) plus the
 * publishing users' links user_ul_tick (user -> broker) and user_dl_tick
 * (broker -> user): [R] (one user per replication, user_per_task = 0) or
 * [R][T] (per task, = 1).  Writes user_stats [R] (device). */
int fognet_user_stats_dev(fognet_ctx *ctx, const fognet_batch_in *in, const fognet_batch_out *out,
                          const int64_t *user_ul_tick, const int64_t *user_dl_tick, int32_t user_per_task,
                          fognet_user_stats *user_stats, void *hip_stream);

/* Exact reduction of R per-replication stats (device pointers) into one job
 * record (device pointer).  Replications with status != OK count in n_failed
 * and contribute nothing else.  R > 4096 reduces through partial records in
 * the context's workspace: reductions on one context must then be enqueued
 * on one stream (or synchronised), since concurrent ones share it. */
int fognet_reduce_stats_dev(fognet_ctx *ctx, const fognet_rep_stats *stats, int32_t R,
                            fognet_job_stats *out, void *hip_stream);
/* Host-side exact merge (used to combine per-GPU records after an all-gather):
 * *acc = *acc (+) *other.  fognet_job_stats_init() sets the identity. */
void fognet_job_stats_init(fognet_job_stats *s);
void fognet_job_stats_merge(fognet_job_stats *acc, const fognet_job_stats *other);
/* Host-side exact accumulate of one replication (what fognet_reduce_stats_dev
 * does per replication; energy is added in call order): for callers of the
 * host-buffer fognet_run_batch. */
void fognet_job_stats_add_rep(fognet_job_stats *acc, const fognet_rep_stats *rep);

/* Device trace generator: fills arrive/req [R][T] and node params [R][N]
 * (replications r0 .. r0+R-1 of the recipe; r0 lets GPUs shard one job). */
int fognet_gen_trace_dev(fognet_ctx *ctx, const fognet_gen_params *p, int64_t r0, int32_t R,
                         int32_t T, int32_t N, int64_t *arrive_tick, int32_t *req_mips,
                         int32_t *mips, int64_t *dl_tick, int64_t *ul_tick, int64_t *init_adv_tick,
                         void *hip_stream);

/* Generated replay ("traces are generated in-kernel ...
 * only stats and histograms are written"): replications r0 .. r0 + R - 1 of
 * the fognet_gen_trace_dev recipe (p; mean_gap_ticks / lat_scale indexed by the
 * local replication 0 .. R-1) are replayed with each 64-publish chunk of the
 * trace and the node parameters computed inside the replay kernel; no trace
 * and no per-task output ever reaches memory.  Results equal
 * fognet_gen_trace_dev + fognet_run_batch_dev on the same replications.
 *   in:  R, T, N, policy, ring_capacity, p_busy_w/p_idle_w, node_stride (and
 *        hier_threshold_s / hier_up_tick for EXT_HIER); every trace/node-parameter
 *        pointer, down_tick and region must be NULL.  EXT_HIER: publish i's regional
 *        broker follows the builder-defined mobility model of the Python mirror's
 *        mobility_regions with its defaults (256 users, user i mod 256 starts in
 *        region (i mod 256) mod B, moves +1 (even) / -1 (odd) every 30/45/60/75 s
 *        (user mod 4) from the first publish), computed in the kernel; EXT_HIER and
 *        replays with T * (req_hi / 1000) >= 2^32 run on the wide kernel.
 *   out: stats [R] (required), hist (added to), node_energy_j (nullable);
 *        node/status/start_tick/done_tick must be NULL. */
int fognet_run_generated_dev(fognet_ctx *ctx, const fognet_gen_params *p, int64_t r0,
                             const fognet_batch_in *in, fognet_batch_out *out, void *hip_stream);

/* Synchronise the context's device. */
int fognet_sync(fognet_ctx *ctx);

/* EXT_HIER with N > 1024 (more than one region), fognet_run_batch[_dev]: the path each
 * launch took (diagnostic).  A launch first replays every (replication, region) pair on
 * its own wavefront and hands a replication with any escalation to the sequential
 * replay, which continues it from its first escalated publish (region_launches); or it
 * runs the sequential replay for every replication (sequential_launches).  Both give
 * identical results.  FOGNET_HIER_REGIONS (environment): unset or "1" -- the region pass;
 * "0" -- always sequential; "only" -- the region pass without the hand-over (testing: a
 * handed-over replication then reports FOGNET_ERR_UNSUPPORTED).  FOGNET_HIER_RESUME=0: the
 * sequential replay restarts a handed-over replication from its first publish, and with
 * FOGNET_HIER_REGIONS unset the path is chosen per launch: while the last region pass
 * whose hand-over count has reached the host (copied back asynchronously, read without
 * waiting) handed more than half of its replications over, the next launches go straight
 * to the sequential replay, with a region pass again every 16th launch to re-measure. */
int fognet_hier_path_stats(const fognet_ctx *ctx, int64_t *region_launches, int64_t *sequential_launches);

/* ---- Multi-GPU statistics exchange over RCCL (xGMI), SURVEY.md §8(b)
 * `fognet_allreduce_stats` and §8(e): replications are sharded over ranks (one
 * process per GPU) and this end-of-run exchange is the only collective.  RCCL
 * is loaded on first use (librccl.so.1; a copy already in the process, e.g.
 * PyTorch's, is reused).  Rank 0 creates the id; the caller moves its bytes to
 * the other ranks (MPI, a shared file, a TCP store ...).  Collective calls:
 * every rank calls fognet_comm_create / fognet_allreduce_stats in the same order. */
#define FOGNET_COMM_ID_BYTES 128
typedef struct fognet_comm fognet_comm;
int fognet_comm_unique_id(uint8_t id[FOGNET_COMM_ID_BYTES]);
int fognet_comm_create(fognet_ctx *ctx, int32_t world, int32_t rank, const uint8_t id[FOGNET_COMM_ID_BYTES],
                       fognet_comm **out);
void fognet_comm_destroy(fognet_comm *comm);
/* *inout (host): this rank's job record in, the job record of all ranks out:
 * the records are all-gathered and merged in rank order with
 * fognet_job_stats_merge, so the result is exact and identical on every rank
 * (energy: fp64 sum in rank order).  hist (device pointer to
 * [FOGNET_HIST_METRICS][FOGNET_HIST_BINS] int64, nullable): summed in place.
 * Enqueued on hip_stream; returns after the exchange completed. */
int fognet_allreduce_stats(fognet_ctx *ctx, fognet_comm *comm, fognet_job_stats *inout, int64_t *hist,
                           void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* FOGNET_HIP_H */
