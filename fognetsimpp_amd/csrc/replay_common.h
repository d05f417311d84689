// replay_common.h — device pieces shared by the two replay kernels:
// replay.hip (N <= 256, node state in VGPRs) and replay_wide.hip (N <= 65,536,
// node state in LDS + HBM).  Tick arithmetic, the FES same-tick rule and the
// exact per-replication statistics accumulator.
#pragma once

#include "internal.h"

namespace fognet {

constexpr int64_t kNever = INT64_MAX;
// Simulated ticks are kept below 2^61 (26.7 days); service seconds enter the
// tick arithmetic clamped (2^22 s in the wide kernel, 255 s in the register
// kernel), so no intermediate of the replay arithmetic can overflow int64.
constexpr int64_t kMaxTick = (int64_t)1 << 61;

// FOGNET_POLICY_EXT_LAT bounds (fognet_hip.h): service saturates at 2^20 s,
// downlinks stay below 2^50 ticks.
constexpr uint32_t kExtSatS = 1u << 20;
constexpr int64_t kExtMaxDl = (int64_t)1 << 50;

// S seconds in ticks: S * 1e12 = (S * 5^12) << 12, one v_mad_u64_u32 + shift.
__device__ __forceinline__ int64_t ticks_of(uint32_t s) {
  static_assert(kTicksPerSecond == 244140625ll << 12, "1e12 ticks per second");
  return (int64_t)(((uint64_t)s * 244140625u) << 12);
}

// s_waitcnt vmcnt(0) (expcnt, lgkmcnt unconstrained) as the builtin, so the
// compiler's wait insertion knows every load issued so far has landed.  Placed
// inside the arm of a branch that loads, it keeps the wait off the other arm: the
// compiler would otherwise wait at the merge (vmcnt(0), which on gfx9 also waits
// for every store issued before), on every path.
__device__ __forceinline__ void sync_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// arrival at tick `a` happens before the completion at `done` of a task with
// service S on a node with downlink latency dl (FES insertion-order rule,
// DESIGN.md §3.3).
// (S is clamped at 2^22 s: dl < 2^61 ticks is below 2^22 s in ticks, so the
// comparison is unchanged and S * 1e12 cannot overflow)
__device__ __forceinline__ bool arrives_before(int64_t a, int64_t done, int64_t dl, uint32_t S) {
  return a < done || (a == done && dl >= (int64_t)min(S, 1u << 22) * kTicksPerSecond);
}

// Separately rounded IEEE double operations.  hipcc contracts a*b+c into an
// FMA by default, and __dmul_rn/__dadd_rn are plain * and + in a header, so
// they fuse too; these carry the pragma themselves.
__device__ __forceinline__ double mul_rn(double a, double b) {
#pragma clang fp contract(off)
  return a * b;
}
__device__ __forceinline__ double add_rn(double a, double b) {
#pragma clang fp contract(off)
  return a + b;
}

// ---------------------------------------------------------------- wave scans
// Inclusive prefix sum (u32) and prefix maximum (i64) over the 64 lanes: DPP
// row shifts, then the row broadcasts.  Lanes outside the scanned range must
// hold the identities (0, INT64_MIN).
__device__ __forceinline__ uint32_t wave_scan_add_u32(uint32_t v) {
  v += dpp_or_u32<0x111, 0xF>(0u, v);  // row_shr:1
  v += dpp_or_u32<0x112, 0xF>(0u, v);  // row_shr:2
  v += dpp_or_u32<0x114, 0xF>(0u, v);  // row_shr:4
  v += dpp_or_u32<0x118, 0xF>(0u, v);  // row_shr:8
  v += dpp_or_u32<0x142, 0xA>(0u, v);  // row_bcast:15
  v += dpp_or_u32<0x143, 0xC>(0u, v);  // row_bcast:31
  return v;
}

// `tmp` carries the DPP destination from level to level: a lane whose source
// is invalid keeps a value of an earlier lane its running maximum covers.
__device__ __forceinline__ int64_t wave_scan_max_i64(int64_t v) {
  int64_t t = INT64_MIN;
#define FOGNET_MAX_LEVEL(C, M)         \
  t = dpp_or_i64<C, M>(t, v);          \
  v = t > v ? t : v;
  FOGNET_MAX_LEVEL(0x111, 0xF)
  FOGNET_MAX_LEVEL(0x112, 0xF)
  FOGNET_MAX_LEVEL(0x114, 0xF)
  FOGNET_MAX_LEVEL(0x118, 0xF)
  FOGNET_MAX_LEVEL(0x142, 0xA)
  FOGNET_MAX_LEVEL(0x143, 0xC)
#undef FOGNET_MAX_LEVEL
  return v;
}

__device__ __forceinline__ int64_t wave_scan_add_i64(int64_t v) {
  v += dpp_or_i64<0x111, 0xF>(0, v);  // row_shr:1
  v += dpp_or_i64<0x112, 0xF>(0, v);  // row_shr:2
  v += dpp_or_i64<0x114, 0xF>(0, v);  // row_shr:4
  v += dpp_or_i64<0x118, 0xF>(0, v);  // row_shr:8
  v += dpp_or_i64<0x142, 0xA>(0, v);  // row_bcast:15
  v += dpp_or_i64<0x143, 0xC>(0, v);  // row_bcast:31
  return v;
}

// ---------------------------------------------------------------- generated mode
// Publishes c0 .. c0 + 63 of a generated replication, task c0 + lane in each
// lane (the gen_kernel recipe, internal.h): tick ca (kNever past T) and
// requirement cr.  carry: the tick before the chunk's first gap (the previous
// chunk's last tick; max_j ul_j + 1 before the first chunk), advanced past the
// chunk.  The gaps' prefix sum is exact integer arithmetic, so the ticks equal
// gen_kernel's block scan.
__device__ __forceinline__ void gen_chunk(const GenRep& g, int c0, int T, int lane, int64_t& carry, int64_t& ca,
                                          int32_t& cr) {
  const int i = c0 + lane;
  int64_t gap = 0;
  int32_t rq = 0;
  if (i < T) gen_task(g, i, gap, rq);
  const int64_t inc = wave_scan_add_i64(gap);
  ca = i < T ? carry + inc : kNever;
  cr = rq;
  carry += readlane_i64(inc, kWave - 1);
}

// ---------------------------------------------------------------- OMNeT++ SimTime
// The reference's signal arithmetic on simtime_t (OMNeT++ 4.6, scale 1e-12;
// fognet_hip.h "Reference signal values"): dbl() = t * 1e-12, SimTime(double)
// and SimTime * double round with toInt64(x) = floor(x + 0.5) and throw
// outside the int64 range.  Every double operation is separately rounded.

// Generated EXT_HIER (fognet_run_generated_dev): the regional broker of publish i
// of a replication under the builder-defined mobility model of
// fognetsimpp_amd.mobility_regions with its defaults (256 users; user u = i mod 256
// starts in region u mod B and moves one region, +1 for even u and -1 for odd u,
// every 30 / 45 / 60 / 75 s (u mod 4) from the replication's first publish t0).
constexpr int kGenHierUsers = 256;
__device__ __forceinline__ int32_t gen_region(int64_t i, int64_t t, int64_t t0, int B) {
  const int64_t u = i % kGenHierUsers;
  const int64_t per = (int64_t)(30 + 15 * (int)(u % 4)) * kTicksPerSecond;
  const int64_t hops = (t - t0) / per;  // (t >= t0: a floor division)
  int64_t reg = (u % B) + ((u % 2) ? -hops : hops);
  reg %= B;
  return (int32_t)(reg < 0 ? reg + B : reg);
}

__device__ __forceinline__ double simtime_dbl(int64_t t) { return mul_rn((double)t, 1e-12); }

// SimTime::toInt64; false where the reference throws cRuntimeError
__device__ __forceinline__ bool simtime_to_int64(double x, int64_t& out) {
  const double f = floor(add_rn(x, 0.5));
  const bool ok = fabs(f) < 0x1p63;
  out = ok ? (int64_t)f : 0;
  return ok;
}

// queueTime (ComputeBrokerApp3.cc:238, 306): the raw simtime_t of
// (simTime() - SimTime(queueStartTime)) * 1000 for a task enqueued at tick a
// (queueStartTime = simTime().dbl()) that starts at tick now.
__device__ __forceinline__ bool qtime_raw(int64_t now, int64_t a, int64_t& raw) {
  int64_t qs;
  simtime_to_int64(mul_rn(1e12, simtime_dbl(a)), qs);  // a < 2^61: in range
  return simtime_to_int64(mul_rn((double)(now - qs), 1000.0), raw);
}

// (simTime() - t0) * 1000 with t0 a simtime_t (mqttApp2.cc:260,272,282)
__device__ __forceinline__ bool ms_raw(int64_t d, int64_t& raw) {
  return simtime_to_int64(mul_rn((double)d, 1000.0), raw);
}

// histogram bin of a raw ms signal: whole part of the recorded double (ms)
// (the bit length of (uint64)v for v >= 1 is v's binary exponent + 1, frexp's e)
__device__ __forceinline__ int hist_bin_raw(int64_t raw) {
  const double v = simtime_dbl(raw);
  if (!(v >= 1.0)) return 0;
  int b;
  (void)frexp(v, &b);
  return b > FOGNET_HIST_BINS - 1 ? FOGNET_HIST_BINS - 1 : b;
}

// ---------------------------------------------------------------- statistics
// Exact per-replication statistics: queueTime (ComputeBrokerApp3.cc:238) over
// queued tasks as the raw values the reference emits, response (done -
// publish arrival, ticks) over all tasks.  Integer sums are bit-identical for
// any summation order, so every kernel that accumulates them writes the same
// record.

struct Acc {
  uint64_t n4, n5, busy;
  uint64_t qs_lo, qs_hi, qq_lo, qq_hi, qq_top, rs_lo, rs_hi, rq_lo, rq_hi;
  int64_t qmin, qmax, rmin, rmax, last;
  uint64_t nqt, nqo;  // queueTime emissions in the moments / lost to simtime overflow
};

// Unsigned 32-bit division by a per-node constant (the node's MIPS) as a
// multiply-high and two shifts (Granlund & Montgomery 1994, Fig. 4.1):
// n / d = (t + ((n - t) >> sh1)) >> sh2 with t = umulhi(m, n), exact for
// every n < 2^32 and d >= 1.  sh = sh1 | sh2 << 8.
struct UDiv {
  uint32_t m, sh;
};

__device__ __forceinline__ UDiv udiv_magic(uint32_t d) {
  const uint32_t l = d <= 1u ? 0u : 32u - (uint32_t)__clz((int)(d - 1u));  // ceil(log2 d)
  const uint32_t m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1u);
  return UDiv{m, (l < 1u ? l : 1u) | ((l > 1u ? l - 1u : 0u) << 8)};
}

__device__ __forceinline__ uint32_t udiv(uint32_t n, UDiv q) {
  const uint32_t t = __umulhi(q.m, n);
  return (t + ((n - t) >> (q.sh & 0xFFu))) >> (q.sh >> 8);
}

// The reference's abort point: the earliest (tick, then task index) queueTime
// emission that overflows (ComputeBrokerApp3.cc:238 throws and nothing up to
// :84-86 catches, so OMNeT++ ends the run there).  Kept apart from Acc so the
// register-bound statistics loops keep their footprint.
struct AbortPt {
  int64_t tick;  // INT64_MAX: none
  int32_t task;  // INT32_MAX: none
};

__device__ __forceinline__ AbortPt abort_none() { return AbortPt{INT64_MAX, INT32_MAX}; }

__device__ __forceinline__ void abort_min(int64_t& tick, int32_t& task, int64_t t, int32_t k) {
  if (t < tick || (t == tick && k < task)) {
    tick = t;
    task = k;
  }
}
__device__ __forceinline__ void abort_min(AbortPt& a, const AbortPt& b) { abort_min(a.tick, a.task, b.tick, b.task); }

// Minimum over the 64 lanes (all active); ticks are >= 0.
__device__ __forceinline__ AbortPt wave_min_abort(AbortPt a) {
  const uint64_t mt = wave_min_u64((uint64_t)a.tick);
  const uint32_t mk = wave_min_u32((uint64_t)a.tick == mt ? (uint32_t)a.task : ~0u);
  return AbortPt{(int64_t)mt, (int32_t)mk};
}

__device__ __forceinline__ Acc acc_identity() {
  Acc a = {};
  a.qmin = a.rmin = INT64_MAX;
  a.qmax = a.rmax = a.last = INT64_MIN;
  return a;
}

__device__ __forceinline__ void add128(uint64_t& lo, uint64_t& hi, uint64_t vlo, uint64_t vhi) {
  const uint64_t o = lo;
  lo += vlo;
  hi += vhi + (lo < o ? 1u : 0u);
}

// v^2 as a 128-bit (lo, hi) from three 32x32 -> 64 products (v = h 2^32 + l:
// v^2 = h^2 2^64 + 2 h l 2^32 + l^2), instead of the 64-bit low product plus
// __umul64hi (about eight quarter-rate multiplies between them).
__device__ __forceinline__ void sq128(uint64_t v, uint64_t& lo, uint64_t& hi) {
  const uint32_t l = (uint32_t)v, h = (uint32_t)(v >> 32);
  const uint64_t ll = (uint64_t)l * l, hl = (uint64_t)h * l, hh = (uint64_t)h * h;
  lo = ll + (hl << 33);
  hi = hh + (hl >> 31) + (lo < ll ? 1u : 0u);
}

__device__ __forceinline__ void add_moment(uint64_t& slo, uint64_t& shi, uint64_t& qlo, uint64_t& qhi,
                                           uint64_t v) {
  add128(slo, shi, v, 0u);
  uint64_t sl, sh;
  sq128(v, sl, sh);
  add128(qlo, qhi, sl, sh);
}

// 192-bit a += (b_lo, b_hi, b_top)
__device__ __forceinline__ void add192(uint64_t& lo, uint64_t& hi, uint64_t& top, uint64_t blo, uint64_t bhi,
                                       uint64_t btop) {
  const uint64_t o = lo;
  lo += blo;
  const uint64_t c0 = lo < o ? 1u : 0u;
  const uint64_t h0 = hi;
  hi += bhi;
  uint64_t c1 = hi < h0 ? 1u : 0u;
  const uint64_t h1 = hi;
  hi += c0;
  c1 += hi < h1 ? 1u : 0u;
  top += btop + c1;
}

// signed value: two's complement 128-bit sum, 192-bit sum of squares
__device__ __forceinline__ void add_moment_signed(uint64_t& slo, uint64_t& shi, uint64_t& qlo, uint64_t& qhi,
                                                  uint64_t& qtop, int64_t v) {
  const uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  add128(slo, shi, (uint64_t)v, v < 0 ? ~(uint64_t)0 : 0u);
  uint64_t sl, sh;
  sq128(m, sl, sh);
  add192(qlo, qhi, qtop, sl, sh, 0u);
}

// one queueTime emission of a task enqueued at tick a, started at tick start;
// false: the emission overflows (the reference throws there: its abort point)
__device__ __forceinline__ bool acc_qtime(uint64_t& qs_lo, uint64_t& qs_hi, uint64_t& qq_lo, uint64_t& qq_hi,
                                          uint64_t& qq_top, int64_t& qmin, int64_t& qmax, uint64_t& nqt,
                                          uint64_t& nqo, int64_t start, int64_t a, uint32_t* hist) {
  int64_t raw;
  if (qtime_raw(start, a, raw)) {
    add_moment_signed(qs_lo, qs_hi, qq_lo, qq_hi, qq_top, raw);
    qmin = min(qmin, raw);
    qmax = max(qmax, raw);
    nqt += 1u;
    if (hist) atomicAdd(&hist[hist_bin_raw(raw)], 1u);
    return true;
  }
  nqo += 1u;
  return false;
}

// the same into an Acc, with the abort point (task: the task's index)
__device__ __forceinline__ void acc_qtime(Acc& acc, AbortPt& ab, int64_t start, int64_t a, int32_t task,
                                          uint32_t* hist) {
  if (!acc_qtime(acc.qs_lo, acc.qs_hi, acc.qq_lo, acc.qq_hi, acc.qq_top, acc.qmin, acc.qmax, acc.nqt, acc.nqo, start,
                 a, hist))
    abort_min(ab.tick, ab.task, start, task);
}

__device__ __forceinline__ void acc_merge(Acc& a, const Acc& b) {
  a.n4 += b.n4;
  a.n5 += b.n5;
  a.busy += b.busy;
  a.nqt += b.nqt;
  a.nqo += b.nqo;
  add128(a.qs_lo, a.qs_hi, b.qs_lo, b.qs_hi);
  add192(a.qq_lo, a.qq_hi, a.qq_top, b.qq_lo, b.qq_hi, b.qq_top);
  add128(a.rs_lo, a.rs_hi, b.rs_lo, b.rs_hi);
  add128(a.rq_lo, a.rq_hi, b.rq_lo, b.rq_hi);
  a.qmin = min(a.qmin, b.qmin);
  a.qmax = max(a.qmax, b.qmax);
  a.rmin = min(a.rmin, b.rmin);
  a.rmax = max(a.rmax, b.rmax);
  a.last = max(a.last, b.last);
}

// One task's contribution: response = done - publish tick t; queued tasks
// (status 4) also their queueTime emission (enqueued at arrival a, started at
// start).  hist: the queueTime histogram row (nullable).  task: its index.
__device__ __forceinline__ void acc_task(Acc& acc, AbortPt& ab, int64_t t, int64_t a, int64_t start, int64_t done,
                                         uint32_t S, uint32_t status, int32_t task, uint32_t* hist) {
  acc.busy += S;
  const int64_t resp = done - t;
  add_moment(acc.rs_lo, acc.rs_hi, acc.rq_lo, acc.rq_hi, (uint64_t)resp);
  acc.rmin = min(acc.rmin, resp);
  acc.rmax = max(acc.rmax, resp);
  acc.last = max(acc.last, done);
  if (status == 4u) {
    acc.n4 += 1u;
    acc_qtime(acc, ab, start, a, task, hist);
  } else {
    acc.n5 += 1u;
  }
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
  return ((uint64_t)hi << 32) | lo;
}

// Butterfly merge over the 64 lanes of a wave: every lane ends with the total.
__device__ __forceinline__ Acc wave_merge(Acc a) {
#pragma unroll 1
  for (int m = kWave / 2; m > 0; m >>= 1) {
    Acc b;
    b.n4 = shfl_xor_u64(a.n4, m);
    b.n5 = shfl_xor_u64(a.n5, m);
    b.busy = shfl_xor_u64(a.busy, m);
    b.qs_lo = shfl_xor_u64(a.qs_lo, m);
    b.qs_hi = shfl_xor_u64(a.qs_hi, m);
    b.qq_lo = shfl_xor_u64(a.qq_lo, m);
    b.qq_hi = shfl_xor_u64(a.qq_hi, m);
    b.qq_top = shfl_xor_u64(a.qq_top, m);
    b.nqt = shfl_xor_u64(a.nqt, m);
    b.nqo = shfl_xor_u64(a.nqo, m);
    b.rs_lo = shfl_xor_u64(a.rs_lo, m);
    b.rs_hi = shfl_xor_u64(a.rs_hi, m);
    b.rq_lo = shfl_xor_u64(a.rq_lo, m);
    b.rq_hi = shfl_xor_u64(a.rq_hi, m);
    b.qmin = (int64_t)shfl_xor_u64((uint64_t)a.qmin, m);
    b.qmax = (int64_t)shfl_xor_u64((uint64_t)a.qmax, m);
    b.rmin = (int64_t)shfl_xor_u64((uint64_t)a.rmin, m);
    b.rmax = (int64_t)shfl_xor_u64((uint64_t)a.rmax, m);
    b.last = (int64_t)shfl_xor_u64((uint64_t)a.last, m);
    acc_merge(a, b);
  }
  return a;
}

// (ref_abort: FOGNET_FLAG_REF_ABORT; S->status already holds the replay's status)
__device__ __forceinline__ void write_rep_stats(fognet_rep_stats* S, const Acc& b, const AbortPt& ab,
                                                bool ref_abort) {
  S->abort_tick = ab.tick;
  S->abort_task = ab.tick == INT64_MAX ? -1 : (int64_t)ab.task;
  if (ref_abort && ab.tick != INT64_MAX && S->status == FOGNET_OK) S->status = FOGNET_REF_ABORTED;
  S->n_queued = (int64_t)b.n4;
  S->n_started = (int64_t)b.n5;
  S->last_tick = b.last;
  S->queue_min_raw = b.qmin;
  S->queue_max_raw = b.qmax;
  S->resp_min_ticks = b.rmin;
  S->resp_max_ticks = b.rmax;
  S->queue_sum_lo = b.qs_lo;
  S->queue_sum_hi = b.qs_hi;
  S->queue_sq_lo = b.qq_lo;
  S->queue_sq_hi = b.qq_hi;
  S->resp_sum_lo = b.rs_lo;
  S->resp_sum_hi = b.rs_hi;
  S->resp_sq_lo = b.rq_lo;
  S->resp_sq_hi = b.rq_hi;
  S->busy_s = (int64_t)b.busy;
  S->energy_j = 0.0;
  S->queue_sq_top = b.qq_top;
  S->n_qtime = (int64_t)b.nqt;
  S->n_qtime_overflow = (int64_t)b.nqo;
}

// ---------------------------------------------------------------- statistics pass
// The statistics pass over the replay outputs (replay.hip's fused epilogue and
// rep_stats_kernel, replay_region.hip's finish kernel).

// Accumulate tasks i = i0, i0 + stride, ... < n of one replication into `a`
// (plus the per-node service seconds s_busy and the histogram s_hist in LDS
// when those statistics are on).  The loads of UNROLL tasks are issued
// before any is used.  dl_of(k): node k's downlink latency.
// kPerTask = false: busy seconds, per-node service and `last` are not
// accumulated per task (the fused epilogue takes them from the node tails).
// ab_tick/ab_task (LDS, one slot per thread, indexed by i0): the abort point
// (replay_common.h AbortPt) is kept there, a read-modify-write only on an
// overflow, which is rare, instead of in registers (the fused epilogue has
// none to spare).
template <int UNROLL, bool kPerTask = true, class DlOf>
__device__ __forceinline__ void stats_accumulate(const ReplayArgs& A, size_t tbase, int n, int i0, int stride, Acc& a,
                                                 unsigned long long* s_busy, uint32_t* s_hist, DlOf dl_of,
                                                 int64_t* ab_tick, int32_t* ab_task) {
  const bool energy = kPerTask && A.p_busy != nullptr;
  const bool hist = A.hist != nullptr;
  for (int ib = i0; ib < n; ib += stride * UNROLL) {
    int64_t t[UNROLL], st0[UNROLL], dn[UNROLL];
    int32_t kk[UNROLL];
    uint32_t stt[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int i = ib + u * stride;
      const size_t o = tbase + (size_t)(i < n ? i : ib);  // past the end: reload task ib (in bounds, unused)
      t[u] = A.arrive[o];
      kk[u] = A.out_node[o];
      stt[u] = A.out_status[o];
      st0[u] = A.out_start[o];
      dn[u] = A.out_done[o];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (ib + u * stride < n) {
        const int32_t k = kk[u];
        const int64_t resp = dn[u] - t[u];
        if constexpr (kPerTask) {
          const uint64_t svc = (uint64_t)(dn[u] - st0[u]) / (uint64_t)kTicksPerSecond;  // whole seconds
          a.busy += svc;
          if (energy) atomicAdd(&s_busy[k], (unsigned long long)svc);
          a.last = max(a.last, dn[u]);
        }
        add_moment(a.rs_lo, a.rs_hi, a.rq_lo, a.rq_hi, (uint64_t)resp);
        a.rmin = min(a.rmin, resp);
        a.rmax = max(a.rmax, resp);
        if (hist) atomicAdd(&s_hist[FOGNET_HIST_BINS + hist_bin(resp)], 1u);
        if (stt[u] == 4u) {  // queueTime emission (ComputeBrokerApp3.cc:238), enqueued at its arrival
          a.n4 += 1u;
          if (!acc_qtime(a.qs_lo, a.qs_hi, a.qq_lo, a.qq_hi, a.qq_top, a.qmin, a.qmax, a.nqt, a.nqo, st0[u],
                         t[u] + dl_of(k), hist ? s_hist : nullptr))
            abort_min(ab_tick[i0], ab_task[i0], st0[u], ib + u * stride);
        } else {
          a.n5 += 1u;
        }
      }
    }
  }
}

// ---------------------------------------------------------------- wide-record advert
// (replay_wide.hip, replay_region.hip) Saturated advertised busy time in the
// 32-bit view of the wide kernels.
constexpr uint32_t kViewBusySat = 0xFFFFFFFFu;

// The advert of node j's head completion reaches the broker (owner lane):
// the view takes busyTime after releaseResource (ComputeBrokerApp3.cc:232,
// :254) = the service of the tasks that reached j before that completion and
// are not done yet, a difference of cumulative sums; the head advances.
// Returns false when the advertised busy time is 2^24 s or more (only the
// EXT_LAT cost cares: its uint64 tick arithmetic needs busy < 2^24).
// h: node j's record (loaded from HBM or the lane's cached copy), updated in place.
// up: FOGNET_POLICY_EXT_HIER's extra hop, which an escalated task (entry pad
// != 0, bit 31 of the record's tl_S for the tail) took before its downlink:
// the same-tick rule compares the arrival's own insertion tick.
// broken: the chain invariant failed (see below; a library bug, never an input).
__device__ __forceinline__ bool apply_wide_advert(WideNode& h, const WideEntry* e, int64_t dl, int64_t ul, int64_t up,
                                             int64_t& nxt_j, uint32_t& busy_j, bool& broken,
                                             uint32_t* walk = nullptr) {
  // the entry after the head, loaded first: for the lane's cached node h is in
  // registers, so this load issues together with the group's view loads
  WideEntry nx{};
  if (h.npend >= 2) {
    nx = e[h.hd_next];
    sync_vm();  // (in this arm: see sync_vm)
    // Chain invariant, checked at every applied advert: with two or more tasks
    // pending, the record's hd_next names the entry whose prev is the head and
    // whose cumulative service is the head's plus its own.  hd_next changes on
    // three paths -- this advert, a push onto a node with exactly one pending
    // task (hd_next := the pushed task) and a multi-task run onto an idle node
    // (hd_next := its second task) -- so any copy of it elsewhere (the round-2
    // experiment kept one in the HBM view, refreshed only where the view is
    // written: here and on a push onto an idle node) goes stale on the second
    // path, and the next advert then advances the head to a wrong entry.
    broken = nx.prev != h.hd || nx.C != h.hd_C + nx.S;
  }
  uint64_t c_arrived = h.hd_C;  // only the completing task itself ...
  if (arrives_before(h.tl_a, h.hd_done, dl + ((h.tl_S >> 31) ? up : 0), h.hd_S)) {
    c_arrived = h.tl_C;  // ... or everything up to the newest task (the common case)
  } else {
    if (walk) *walk += 1u;  // (profile builds: backward walks, and their steps << 16)
    for (int32_t x = e[h.tl].prev; x != h.hd;) {  // newest first
      if (walk) *walk += 1u << 16;
      const WideEntry ex = e[x];
      if (arrives_before(ex.a, h.hd_done, dl + (ex.pad ? up : 0), h.hd_S)) {
        c_arrived = ex.C;
        break;
      }
      x = ex.prev;
    }
    sync_vm();
  }
  const uint64_t busy = c_arrived - h.hd_C;
  // the view keeps 32 bits, saturated: a saturated node can only be chosen when the
  // decision's minimum itself is saturated, which the decision refuses (kViewBusySat)
  busy_j = busy < (uint64_t)kViewBusySat ? (uint32_t)busy : kViewBusySat;
  h.npend -= 1;
  if (h.npend == 0) {
    nxt_j = kNever;
  } else {
    // FIFO: the next task started at max(arrival, this completion); its
    // done tick was fixed when it was pushed
    h.hd = h.hd_next;
    h.hd_done = nx.done;
    h.hd_C = nx.C;
    h.hd_S = nx.S;
    h.hd_next = nx.next;  // valid while npend >= 2
    nxt_j = nx.done == kNever ? kNever : nx.done + ul;  // never: crashed before it completes
  }
  return busy < ((uint64_t)1 << 24);  // FOGNET_POLICY_EXT_LAT's cost needs busy < 2^24
}

// ---------------------------------------------------------------- a11 energy over node records
// E_j = P_busy_j * B_j + P_idle_j * ((H - B_j 1e12) / 1e12) with B_j = node j's service seconds
// (its tail's cumulative sum, tl_C), each operation separately rounded, summed in node
// order (0, 1, ..., N-1) by one wavefront (all 64 lanes active; the sum is returned in every
// lane).  kDepth chunks of 64 nodes have their loads issued before the first of them is summed:
// the sum is one dependent chain, so the record and power loads must not each wait in it.  Each
// chunk's 64 terms go through LDS (s_buf: 64 doubles of the caller's) and are read back by every
// lane at the same address (a broadcast, 16 at a time), so the chain is a run of fp64 adds on
// VGPRs; taking each term with v_readlane put an SGPR hand-off into every add (~80 cycles per
// node at C5's 10,000 nodes).
template <int kDepth = 8>
// tlc: node j's service seconds at tlc[j * stride] (the records' tl_C: stride 8 over WideNode;
// the region pass's compact tails: stride 2).
__device__ __forceinline__ double energy_sum_wave(const uint64_t* tlc, int stride, const double* p_busy,
                                                  const double* p_idle, int N, int64_t H, double* out_row, int lane,
                                                  double* s_buf) {
  double sum = 0.0;
  for (int c0 = 0; c0 < N; c0 += kDepth * kWave) {
    double en[kDepth];
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int j = c0 + u * kWave + lane;
      en[u] = 0.0;
      if (j < N) {
        const int64_t B = (int64_t)tlc[(size_t)j * (size_t)stride];
        const double eb = mul_rn(p_busy[j], (double)B);
        const double idle = __ddiv_rn((double)(H - B * kTicksPerSecond), 1e12);
        en[u] = add_rn(eb, mul_rn(p_idle[j], idle));
        if (out_row) out_row[j] = en[u];
      }
    }
#pragma unroll
    for (int u = 0; u < kDepth; ++u) {
      const int j0 = c0 + u * kWave;
      const int m = min(kWave, N - j0);
      if (m <= 0) break;
      s_buf[lane] = en[u];
      // every lane's term is in LDS before any lane reads the chunk (one wavefront)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
      if (m == kWave) {
#pragma unroll
        for (int q = 0; q < kWave; q += 16) {
          double v[16];
#pragma unroll
          for (int k = 0; k < 16; ++k) v[k] = s_buf[q + k];
#pragma unroll
          for (int k = 0; k < 16; ++k) sum = add_rn(sum, v[k]);
        }
      } else {
        for (int l = 0; l < m; ++l) sum = add_rn(sum, s_buf[l]);
      }
      // the chunk's reads are done before the next chunk's writes
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
  }
  return sum;
}

}  // namespace fognet
