/*
 * fognet_io.h — host-side formats on either side of the offload-decision path
 * (SURVEY.md §8(f) rows 1 and 3).  Pure host C++ in libfognet_hip: no GPU and
 * no fognet_ctx needed, so an OMNeT++ build, a trace exporter or a CPU test
 * can call these without a device.
 *
 *   - Binary SoA trace files ("FOGNTRC1"): the inputs of fognet_run_batch
 *     (node parameters in CONNECT order + the broker-side publish trace), so
 *     the same bytes feed the GPU engine, the CPU oracle and a reference run.
 *   - OMNeT++ 4.6 result files: `.sca` (scalar/statistic/field/bin lines as in
 *     simulations/example/results/General-0.sca:4957-4967) and `.vec`
 *     (vector declarations + data lines, General-0.vec / General-0.vci) from
 *     the engine's job record, histogram and per-task outputs.
 *   - The reference's task source, mqttApp2::sendMqttData
 *     (src/mqttapp/mqttApp2.cc:353-409): glibc rand() stream shared by every
 *     user in event order, MIPSRequired = 200 + rand() % 701.
 *
 * Errors: fognet_status codes (fognet_hip.h); the message of the last failure
 * on the calling thread is fognet_io_last_error().
 */
#ifndef FOGNET_IO_H
#define FOGNET_IO_H

#include <stdint.h>

#include "fognet_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define FOGNET_TRACE_MAGIC "FOGNTRC1"
#define FOGNET_TRACE_VERSION 1
#define FOGNET_TRACE_HEADER_BYTES 256
#define FOGNET_TRACE_ALIGN 64

/* Trace file layout (little endian):
 *   header (FOGNET_TRACE_HEADER_BYTES): magic[8], u32 version, u32 header_bytes,
 *     i32 R, T, N, node_stride (0: node parameters shared, N: one row per
 *     replication), u32 flags, u32 reserved, u64 payload_bytes, u64 checksum
 *     (FNV-1a 64 over the payload), char note[FOGNET_TRACE_NOTE_BYTES]
 *     (free text, NUL padded), zero padding;
 *   payload, each section starting at a multiple of FOGNET_TRACE_ALIGN from
 *     the file start, in this order (NR = node_stride ? R : 1):
 *     mips i32 [NR][N], dl_tick i64 [NR][N], ul_tick i64 [NR][N],
 *     init_adv_tick i64 [NR][N], node_id i32 [NR][N] (flag NODE_ID),
 *     p_busy_w f64 [NR][N], p_idle_w f64 [NR][N] (flag POWER),
 *     arrive_tick i64 [R][T], req_mips i32 [R][T]. */
#define FOGNET_TRACE_NOTE_BYTES 160
#define FOGNET_TRACE_FLAG_POWER 1u    /* p_busy_w / p_idle_w sections present            */
#define FOGNET_TRACE_FLAG_NODE_ID 2u  /* node_id section present (module ids, .sca names) */

typedef struct fognet_trace_info {
    int32_t R, T, N, node_stride;
    uint32_t flags;
    uint32_t version;
    uint64_t payload_bytes;
    uint64_t checksum;
    char note[FOGNET_TRACE_NOTE_BYTES];
} fognet_trace_info;

const char *fognet_io_last_error(void);

/* Write in (host pointers; policy and ring_capacity are not stored) to path.
 * node_id: [NR][N] module ids (nullable: not stored).  note: nullable. */
int fognet_trace_write(const char *path, const fognet_batch_in *in, const int32_t *node_id, const char *note);

/* Read and validate the header (magic, version, sizes, file length). */
int fognet_trace_info_read(const char *path, fognet_trace_info *info);

/* Read the whole trace into caller buffers sized from fognet_trace_info:
 * out->arrive_tick .. init_adv_tick are required; out->p_busy_w/p_idle_w
 * and node_id are filled when non-null and present (FOGNET_ERR_ARG when
 * non-null but absent).  R/T/N/node_stride of *out are set from the file.
 * The checksum is verified (FOGNET_ERR_ARG on mismatch). */
int fognet_trace_read(const char *path, fognet_batch_in *out, int32_t *node_id);

/* OMNeT++ .sca of one job record.  run_id: "run" line (e.g.
 * "General-0-20260101-00:00:00-1"); network: module path prefix (e.g.
 * "FogNet").  Writes, under <network>.broker.udpApp[0] and
 * <network>.fogNodes.udpApp[0]: scalars (decisions, queued, started,
 * replications, failed replications, busy seconds, energy J, makespan s),
 * `queueTime:stats` and `response:stats` (ms; count/mean/stddev/sum/sqrsum/
 * min/max computed from the exact integer sums, printed %.14g like
 * OMNeT++), and when hist != NULL `queueTime:histogram` /
 * `response:histogram` with the FOGNET_HIST_BINS bins (lower bound ms). */
int fognet_write_sca(const char *path, const char *run_id, const char *network, const fognet_job_stats *job,
                     const int64_t *hist /* [FOGNET_HIST_METRICS][FOGNET_HIST_BINS], nullable */);

/* OMNeT++ .vec of one replication's per-task outputs (host arrays of length
 * T): vector `queueTime:vector` of every fog node module
 * <network>.fogNode[<node_id or index>].udpApp[0] (value ms, emitted at the
 * task's service start, queued tasks only: ComputeBrokerApp3.cc:238) and
 * `decision:vector` of <network>.broker.udpApp[0] (chosen node index at the
 * publish tick).  Columns "TV" (time, value): the engine has no OMNeT++ event
 * numbers.  Times print as exact decimal seconds (12 fractional digits,
 * trailing zeros trimmed).  node_id: nullable (index names). */
int fognet_write_vec(const char *path, const char *run_id, const char *network, int32_t T, int32_t N,
                     const int64_t *arrive_tick, const int64_t *dl_tick /* [N] */, const int32_t *node,
                     const uint8_t *status, const int64_t *start_tick, const int32_t *node_id);

/* The reference task source (mqttApp2.cc:198-409 with the ini keys of
 * simulations/example/wirelessNet.ini:48-52), restated as a small event
 * simulation of U users and the broker's CONNECT handling:
 *   START(u) at start_tick[u] (mqttApp2::processStart/processSend): sends
 *     CONNECT (reaches the broker at +uplink_tick[u]) and arms the MQTTDATA
 *     timer at start + interval_tick[u] (if < stop_tick);
 *   CONNECT at the broker (BrokerBaseApp3.cc:99-121): the CONNACK reaches
 *     the user downlink_tick[u] later (downlink_tick[u] < 0: never);
 *   CONNACK at the user (processConSubAck, :319-325): publishes at once;
 *   MQTTDATA (sendMqttData, :353-409): publishes.
 * A publish draws MIPSRequired = req_base + rand() % req_span from ONE glibc
 * rand() stream seeded by srand(seed) (the TYPE_3 additive feedback
 * generator of glibc random_r.c, shared by every user in event order) and,
 * if now + interval < stop_tick, cancels and re-arms the user's timer at
 * now + interval.  Events are processed in OMNeT++ FES order (tick,
 * insertion sequence); the START events are inserted first, in user order.
 * Each publish reaches the broker uplink_tick[u] after it is sent; the trace
 * is ordered by (broker arrival tick, send order), the broker's FES order.
 * Writes at most cap publishes; *out_T = publishes generated
 * (FOGNET_ERR_CAPACITY if > cap, with the first cap written).  user_of
 * (nullable): publishing user of each trace entry. */
int fognet_gen_trace_mqtt(uint32_t seed, int32_t U, const int64_t *start_tick, const int64_t *interval_tick,
                          const int64_t *uplink_tick, const int64_t *downlink_tick, int64_t stop_tick,
                          int32_t req_base, int32_t req_span, int32_t cap, int64_t *arrive_tick,
                          int32_t *req_mips, int32_t *user_of, int32_t *out_T);

#ifdef __cplusplus
}
#endif
#endif /* FOGNET_IO_H */
