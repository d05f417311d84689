// replay.hip — batched trace replay of FogNetSim++'s offload-decision loop on
// gfx950.  One wavefront replays one replication; each lane owns up to four
// fog nodes (node k -> lane k % 64, slot k / 64) whose state lives in VGPRs.
//
// Reference semantics restated (paths relative to the FogNetSim++ tree):
//   decision   BrokerBaseApp3::sendPubAck(status=false)   BrokerBaseApp3.cc:265-304
//   arrival    ComputeBrokerApp3::processPacket (task)     ComputeBrokerApp3.cc:269-320
//   completion ComputeBrokerApp3::releaseResource          ComputeBrokerApp3.cc:224-256
//   advert     ComputeBrokerApp3::advertiseMIPS + broker   ComputeBrokerApp3.cc:205-222,
//              view update                                 BrokerBaseApp3.cc:123-130
//
// Instead of dispatching the ~4 FES events per task one by one, the kernel
// walks the broker's publishes in trace order and derives everything else in
// closed form (DESIGN.md §Replay algorithm):
//   * a node is a FIFO single server, so a task's service start/done ticks
//     follow from the previous task on the same node when it is decided;
//   * the broker's view of node k changes only when the advert of one of k's
//     completions arrives (done + ul_k); adverts that land strictly before a
//     publish's tick are applied before that publish is decided;
//   * the busyTime an advert carries is the service time of the tasks that
//     reached the node before that completion and are not done yet, i.e. a
//     difference of two cumulative sums over the node's pending-task ring;
//   * same-tick ordering follows OMNeT++'s (tick, insertion order) FES rule:
//     trace publishes precede dynamic events at their tick, and a task's
//     arrival precedes a same-tick completion iff dl_k >= S_completing * 1e12.
#include "internal.h"

namespace fognet {

namespace {

struct Slot {
  uint64_t vkey;     // broker view of the node: (advertised busy seconds << 16) | node index
  int64_t nxt;       // tick at which the head's completion advert reaches the broker
  int64_t hd_done;   // head (oldest pending) task: completion tick
  uint32_t hd_C;
  uint32_t hd_S;      // head service seconds (bits 0-23) | nh prefetch stamp (bits 24-31)
  u32x4 nh;          // entry head+1 as loaded {a lo, a hi, C, S} (valid when >= 2 pending)
  int64_t tl_a;      // tail (newest) task
  int64_t tl_done;
  uint32_t tl_C, tl_S;
  uint32_t cnt;      // ring counters mod 2^16: tasks ever assigned (bits 0-15),
                     // completion adverts applied (bits 16-31); capacity <= 2^15
};

// ---- head+1 prefetch, outside the compiler's wait-count tracking
//
// The head+1 entry of a node is needed at that node's next advert, typically
// many publishes later.  A compiler-visible load cannot express that: its
// loop-carried destination gets a conservative `s_waitcnt vmcnt(0)` at the
// first read in the next loop iteration (loads and stores share the in-order
// vmcnt counter, and the count between issue and use is data dependent).  So
// the prefetch is an inline-asm load into the tied loop-carried registers,
// and reads are preceded by an explicit wait (nh_read_*) whose count follows
// from the publishes decided since the issue: each publish issues >= 5 vector
// memory operations (one ring store, four output stores), so a load issued
// >= kPrefetchAge publishes ago is older than the kPrefetchOps youngest and has
// completed once vmcnt <= kPrefetchOps.  Vector-memory loads return in issue
// order on gfx950, so a newer prefetch into the same registers wins.
constexpr uint32_t kPrefetchAge = 8;
constexpr int kPrefetchOps = 40;  // 5 * kPrefetchAge, <= 63 (vmcnt field)

__device__ __forceinline__ void prefetch_entry(u32x4& nh, const RingEntry* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "+v"(nh) : "v"(p) : "memory");
}

// Wave-level wait, then copy nh into fresh registers in the same asm
// statement, so no compiler-generated instruction ever reads nh: the
// registers are only named by these asm statements (an input operand is read
// in place; a tied "+v" operand would be copied around the asm).
#define FOGNET_NH_READ(CNT)                                                                          \
  __device__ __forceinline__ u32x4 nh_read_##CNT(const u32x4& nh) {                                  \
    uint32_t x, y, z, w;                                                                             \
    asm volatile("s_waitcnt vmcnt(" #CNT ")\n\tv_mov_b32 %0, %4\n\tv_mov_b32 %1, %5\n\t"             \
                 "v_mov_b32 %2, %6\n\tv_mov_b32 %3, %7"                                              \
                 : "=&v"(x), "=&v"(y), "=&v"(z), "=&v"(w)                                            \
                 : "v"(nh.x), "v"(nh.y), "v"(nh.z), "v"(nh.w));                                      \
    return u32x4{x, y, z, w};                                                                        \
  }
FOGNET_NH_READ(0)
FOGNET_NH_READ(40)
#undef FOGNET_NH_READ
static_assert(kPrefetchOps == 40, "nh_read_40 encodes the count");

__device__ __forceinline__ uint32_t n_push(const Slot& st) { return st.cnt & 0xFFFFu; }
__device__ __forceinline__ uint32_t n_head(const Slot& st) { return st.cnt >> 16; }
__device__ __forceinline__ uint32_t pending(const Slot& st) { return (n_push(st) - n_head(st)) & 0xFFFFu; }

__device__ __forceinline__ uint32_t head_S(const Slot& st) { return st.hd_S & 0xFFFFFFu; }
// 8-bit issue stamp of the node's pending prefetch; a wrapped stamp can only
// make an old prefetch look recent (a full wait), never the reverse.
__device__ __forceinline__ void stamp_prefetch(Slot& st, uint32_t tix) {
  st.hd_S = (st.hd_S & 0xFFFFFFu) | (tix << 24);
}
__device__ __forceinline__ uint32_t prefetch_age(const Slot& st, uint32_t tix) {
  return (tix - (st.hd_S >> 24)) & 0xFFu;
}

constexpr uint64_t kNoKey = ~0ull;
constexpr int64_t kNever = INT64_MAX;

__device__ __forceinline__ int64_t nh_a(u32x4 v) { return (int64_t)(((uint64_t)v.y << 32) | v.x); }

// arrival at tick `a` happens before the completion at `done` of a task with
// service S on a node with downlink latency dl (FES insertion-order rule).
__device__ __forceinline__ bool arrives_before(int64_t a, int64_t done, int64_t dl, uint32_t S) {
  return a < done || (a == done && dl >= (int64_t)S * kTicksPerSecond);
}

// Apply the advert of the head completion of node k (lane-local).  nhw is
// st.nh read after the wait (nh_read_*).  tix: index of the publish being decided.
__device__ __forceinline__ void apply_advert(Slot& st, const u32x4 nhw, int k, int64_t dl, int64_t ul,
                                             const RingEntry* ring, uint32_t qmask, uint32_t tix) {
  // Cumulative service of the tasks that reached the node before the head's
  // completion: scan back from the newest assignment.
  uint32_t c_arrived = st.hd_C;  // the head itself always arrived before it completed
  const uint32_t pend0 = pending(st);  // >= 1 whenever an advert is due
  if (arrives_before(st.tl_a, st.hd_done, dl, head_S(st))) {
    c_arrived = st.tl_C;
  } else {
    // entries head+d, d = pend0-2 .. 1 (the tail, d = pend0-1, did not qualify)
    for (uint32_t d = pend0 - 1u; d-- > 1u;) {
      int64_t a;
      uint32_t C;
      if (d == 1u) {
        a = nh_a(nhw);
        C = nhw.z;
      } else {
        const RingEntry e = ring[(n_head(st) + d) & qmask];
        a = e.a;
        C = e.C;
      }
      if (arrives_before(a, st.hd_done, dl, head_S(st))) {
        c_arrived = C;
        break;
      }
    }
  }
  const uint32_t busy = c_arrived - st.hd_C;  // busyTime after releaseResource (:232, :254)
  st.vkey = ((uint64_t)busy << 16) | (uint32_t)k;

  // advance the head
  st.cnt += 0x10000u;
  const uint32_t pend = pending(st);
  if (pend == 0u) {
    st.nxt = kNever;
    return;
  }
  const int64_t na = nh_a(nhw);
  const int64_t start = na > st.hd_done ? na : st.hd_done;
  st.hd_done = start + (int64_t)nhw.w * kTicksPerSecond;
  st.hd_C = nhw.z;
  st.hd_S = (st.hd_S & 0xFF000000u) | nhw.w;
  st.nxt = st.hd_done + ul;
  if (pend >= 2u) {  // the ring holds every pending entry, the tail included
    prefetch_entry(st.nh, ring + ((n_head(st) + 1u) & qmask));
    stamp_prefetch(st, tix);
  }
}

// Reload nh of every lane in a slot from its node's current head+1 ring entry,
// issued by all lanes in uniform control flow (an asm load inside a divergent
// branch is given a temporary that the compiler copies back before the data
// lands).  For a lane whose head+1 did not change this is a duplicate of the
// same address: the register already holds, or will receive, the same value,
// so its stamp is left alone.  The ring store of a just-pushed entry precedes
// this load in the same lane, which therefore observes it.
__device__ __forceinline__ void refill_slot(Slot& st, const RingEntry* ring, uint32_t qmask) {
  prefetch_entry(st.nh, ring + ((n_head(st) + 1u) & qmask));
}

// Assign publish o_idx, decided at tick t with requirement rq, to node k
// (lane-local).  Returns (fognet_status << 24) | tasks pending on k after the push.
__device__ __forceinline__ uint32_t push_task(Slot& st, int k, int64_t t, int32_t rq, int64_t dl, int64_t ul,
                                              int32_t mips, RingEntry* ring, uint32_t qmask,
                                              const ReplayArgs& A, size_t o_idx, uint32_t tix) {
  const uint32_t max_s = A.max_s;
  struct {
    uint32_t err;
  } o;
  o.err = FOGNET_OK;
  const uint32_t S = (uint32_t)rq / (uint32_t)mips;  // double tskTime = requiredMIPS / MIPS (:276)
  const int64_t dur = (int64_t)S * kTicksPerSecond;
  if (S > max_s || t > kNever - dl) o.err = FOGNET_ERR_ARG;
  const int64_t a = t + dl;
  uint32_t status;
  int64_t start;
  if (st.tl_done < a) {  // tl_done starts at INT64_MIN: first task of the node
    status = 5u;  // idle: "task assigned" (:282-301)
    start = a;
  } else if (st.tl_done > a) {
    status = 4u;  // busy: "task queued" (:304-313), starts when the previous one completes
    start = st.tl_done;
  } else {  // completion of the previous task at the same tick
    status = (dl < (int64_t)st.tl_S * kTicksPerSecond) ? 5u : 4u;
    start = a;
  }
  if (start > kNever - dur) o.err = FOGNET_ERR_ARG;
  const int64_t done = start + dur;
  if (done > kNever - ul) o.err = FOGNET_ERR_ARG;
  const uint32_t pend = pending(st);
  if (pend > qmask) o.err = FOGNET_ERR_CAPACITY;
  const uint32_t C = st.tl_C + S;
  if (o.err == FOGNET_OK) {
    RingEntry e;
    e.a = a;
    e.C = C;
    e.S = S;
    RingEntry* slot = ring + (n_push(st) & qmask);
    *slot = e;
    if (pend == 0u) {
      st.hd_done = done;
      st.hd_C = C;
      st.hd_S = (st.hd_S & 0xFF000000u) | S;
      st.nxt = done + ul;
    } else if (pend == 1u) {
      // the new entry is head+1: the caller reloads nh for the whole slot
      // (refill_slot), in uniform control flow
      stamp_prefetch(st, tix);
    }
    st.tl_a = a;
    st.tl_C = C;
    st.tl_S = S;
    st.tl_done = done;
    st.cnt = (st.cnt & 0xFFFF0000u) | ((st.cnt + 1u) & 0xFFFFu);
    // per-task outputs, stored by the owner lane (consecutive tasks write
    // consecutive addresses; the partial lines merge in L2)
    A.out_node[o_idx] = k;
    A.out_status[o_idx] = (uint8_t)status;
    A.out_start[o_idx] = start;
    A.out_done[o_idx] = done;
  }
  return (o.err << 24) | (pend + 1u);
}

template <int NPL>
__device__ __forceinline__ uint64_t view_min(const Slot (&st)[NPL]) {
  uint64_t m = st[0].vkey;
#pragma unroll
  for (int s = 1; s < NPL; ++s) m = umin64(m, st[s].vkey);
  return wave_min_u64(m);
}

template <int NPL>
// 4 waves per SIMD (<= 128 VGPRs): 16 replications resident per CU, so the
// 4096-replication sweep runs in a single wave of workgroups on 256 CUs.
__global__ __launch_bounds__(64, 4) void replay_kernel(ReplayArgs A) {
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  __shared__ int64_t s_dl[NPL * kWave];
  __shared__ int64_t s_ul[NPL * kWave];
  __shared__ int32_t s_mips[NPL * kWave];

  const int T = A.T, N = A.N;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  const uint32_t qmask = (1u << A.q_log2) - 1u;
  const int64_t arrive0 = T > 0 ? A.arrive[tbase] : kNever;

  // ---- node parameters + preconditions (fognet_hip.h, fognet_batch_in)
  bool bad = false;
  Slot st[NPL];
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const int k = s * kWave + lane;
    int64_t d = 0, u = 0;
    int32_t m = 1;
    if (k < N) {
      m = A.mips[nbase + k];
      d = A.dl[nbase + k];
      u = A.ul[nbase + k];
      const int64_t ia = A.init[nbase + k];
      bad |= (m <= 0) | (d < 0) | (u < 0) | (ia < u) | (ia >= arrive0);
    }
    s_dl[k] = d;
    s_ul[k] = u;
    s_mips[k] = m;
    // every node's first advert {MIPS, busyTime = 0.0} has reached the broker
    st[s].vkey = k < N ? (uint64_t)k : kNoKey;
    st[s].nxt = kNever;
    st[s].hd_done = 0;
    st[s].hd_C = 0u;
    st[s].hd_S = 0u;
    st[s].nh = u32x4{0u, 0u, 0u, 0u};
    st[s].tl_a = 0;
    st[s].tl_done = INT64_MIN;
    st[s].tl_C = 0u;
    st[s].tl_S = 0u;
    st[s].cnt = 0u;
  }
  __syncthreads();

  uint32_t err = ballot(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;
  if (N <= 0) err = FOGNET_ERR_NO_NODES;

  RingEntry* const ring_r = A.ring + (size_t)r * (size_t)N * ((size_t)qmask + 1u);
  // ring of this lane's node in slot s (lanes past N alias node 0: in bounds,
  // never used); recomputed at each use rather than held in 2 VGPRs per slot
  const int q_log2 = A.q_log2;
  auto ring_s = [&](int s) -> RingEntry* {
    const int k = s * kWave + lane;
    return ring_r + ((size_t)(k < N ? k : 0) << q_log2);
  };
  uint64_t best = view_min<NPL>(st);
  bool dirty = false;
  int64_t prev_t = INT64_MIN;
  uint32_t max_pend = 0u;
  int64_t n_done = 0;

  for (int c0 = 0; c0 < T && err == FOGNET_OK; c0 += kWave) {
    const int cnt = min(kWave, T - c0);
    const bool live = lane < cnt;
    const int64_t ca = live ? A.arrive[tbase + c0 + lane] : kNever;
    const int32_t cr = live ? A.req[tbase + c0 + lane] : 0;
    // trace preconditions: nondecreasing ticks, requirement >= 0
    const int64_t up = (int64_t)(((uint64_t)(uint32_t)__shfl_up((int)((uint64_t)ca >> 32), 1) << 32) |
                                 (uint32_t)__shfl_up((int)(uint32_t)(uint64_t)ca, 1));
    const int64_t prv = lane == 0 ? prev_t : up;
    if (ballot(live && (ca < prv || cr < 0))) {
      err = FOGNET_ERR_ARG;
      break;
    }
    prev_t = readlane_i64(ca, cnt - 1);

    int j = 0;
    for (; j < cnt; ++j) {
      const int64_t t = readlane_i64(ca, j);
      const int32_t rq = (int32_t)readlane_u32((uint32_t)cr, j);
      const uint32_t tix = (uint32_t)(c0 + j);

      // 1) completion adverts that reached the broker strictly before t
#pragma unroll
      for (int s = 0; s < NPL; ++s) {
        for (;;) {
          const bool due = st[s].nxt < t;
          if (!ballot(due)) break;
          dirty = true;
          // the due nodes read their prefetched head+1 entry
          u32x4 nhw;
          if (ballot(due && prefetch_age(st[s], tix) < kPrefetchAge)) {
            nhw = nh_read_0(st[s].nh);
          } else {
            nhw = nh_read_40(st[s].nh);
          }
          if (due) {
            const int k = s * kWave + lane;
            apply_advert(st[s], nhw, k, s_dl[k], s_ul[k], ring_s(s), qmask, tix);
          }
        }
      }
      // 2) argmin over the advertised view (ties -> lowest index)
      if (dirty) {
        best = view_min<NPL>(st);
        dirty = false;
      }
      const int k = (int)(best & 0xFFFFull);
      const int ks = k / kWave, kl = k % kWave;
      // 3) the chosen node receives the task
      uint32_t po = 0u;
#pragma unroll
      for (int s = 0; s < NPL; ++s) {
        if (s == ks && lane == kl) {
          po = push_task(st[s], k, t, rq, s_dl[k], s_ul[k], s_mips[k], ring_s(s), qmask, A,
                         tbase + c0 + j, tix);
        }
      }
      const uint32_t pr = readlane_u32(po, kl);
      if ((pr >> 24) != 0u) {
        err = pr >> 24;
        break;
      }
      const uint32_t pend = pr & 0xFFFFFFu;
      max_pend = pend > max_pend ? pend : max_pend;
      if (pend == 2u) {  // the new entry became head+1 of node k
#pragma unroll
        for (int s = 0; s < NPL; ++s)
          if (s == ks) refill_slot(st[s], ring_s(s), qmask);
      }
    }
    n_done += j;
  }
  // drain the inline-asm prefetches before the wave retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (lane == 0 && A.out_stats) {
    fognet_rep_stats* S = A.out_stats + r;
    S->n_tasks = n_done;
    S->max_pending = (int32_t)max_pend;
    S->status = (int32_t)err;
    S->events = 2 * (int64_t)N + 4 * n_done;
  }
}

// ---------------------------------------------------------------- statistics
// Exact per-replication statistics from the replay outputs: queueTime
// (ComputeBrokerApp3.cc:238) over queued tasks, response (done - publish
// arrival) over all tasks.  128-bit integer sums: bit-identical for any
// summation order.

struct Acc {
  uint64_t n4, n5;
  uint64_t qs_lo, qs_hi, qq_lo, qq_hi, rs_lo, rs_hi, rq_lo, rq_hi;
  int64_t qmin, qmax, rmin, rmax, last;
};

__device__ __forceinline__ void add128(uint64_t& lo, uint64_t& hi, uint64_t vlo, uint64_t vhi) {
  const uint64_t o = lo;
  lo += vlo;
  hi += vhi + (lo < o ? 1u : 0u);
}

__device__ __forceinline__ void add_moment(uint64_t& slo, uint64_t& shi, uint64_t& qlo, uint64_t& qhi,
                                           uint64_t v) {
  add128(slo, shi, v, 0u);
  add128(qlo, qhi, v * v, __umul64hi(v, v));
}

__device__ __forceinline__ void acc_merge(Acc& a, const Acc& b) {
  a.n4 += b.n4;
  a.n5 += b.n5;
  add128(a.qs_lo, a.qs_hi, b.qs_lo, b.qs_hi);
  add128(a.qq_lo, a.qq_hi, b.qq_lo, b.qq_hi);
  add128(a.rs_lo, a.rs_hi, b.rs_lo, b.rs_hi);
  add128(a.rq_lo, a.rq_hi, b.rq_lo, b.rq_hi);
  a.qmin = min(a.qmin, b.qmin);
  a.qmax = max(a.qmax, b.qmax);
  a.rmin = min(a.rmin, b.rmin);
  a.rmax = max(a.rmax, b.rmax);
  a.last = max(a.last, b.last);
}

constexpr int kStatThreads = 256;

__global__ __launch_bounds__(kStatThreads) void rep_stats_kernel(ReplayArgs A) {
  const int r = blockIdx.x;
  __shared__ Acc s_acc[kStatThreads];
  fognet_rep_stats* S = A.out_stats + r;
  const int32_t n = (int32_t)S->n_tasks;  // written by replay_kernel
  const size_t tbase = (size_t)r * (size_t)A.T;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  Acc a = {};
  a.qmin = a.rmin = INT64_MAX;
  a.qmax = a.rmax = a.last = INT64_MIN;
  for (int i = threadIdx.x; i < n; i += kStatThreads) {
    const int64_t t = A.arrive[tbase + i];
    const int32_t k = A.out_node[tbase + i];
    const uint8_t stt = A.out_status[tbase + i];
    const int64_t st0 = A.out_start[tbase + i];
    const int64_t dn = A.out_done[tbase + i];
    const int64_t resp = dn - t;
    add_moment(a.rs_lo, a.rs_hi, a.rq_lo, a.rq_hi, (uint64_t)resp);
    a.rmin = min(a.rmin, resp);
    a.rmax = max(a.rmax, resp);
    a.last = max(a.last, dn);
    if (stt == 4) {
      const int64_t q = st0 - (t + A.dl[nbase + k]);
      a.n4 += 1u;
      add_moment(a.qs_lo, a.qs_hi, a.qq_lo, a.qq_hi, (uint64_t)q);
      a.qmin = min(a.qmin, q);
      a.qmax = max(a.qmax, q);
    } else {
      a.n5 += 1u;
    }
  }
  s_acc[threadIdx.x] = a;
  __syncthreads();
  for (int w = kStatThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) acc_merge(s_acc[threadIdx.x], s_acc[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const Acc& b = s_acc[0];
    S->n_queued = (int64_t)b.n4;
    S->n_started = (int64_t)b.n5;
    S->last_tick = b.last;
    S->queue_min_ticks = b.qmin;
    S->queue_max_ticks = b.qmax;
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
  }
}

}  // namespace

hipError_t launch_replay(const ReplayArgs& a, hipStream_t s) {
  const int npl = (a.N + kWave - 1) / kWave;
  if (npl <= 1) {
    hipLaunchKernelGGL(replay_kernel<1>, dim3(a.R), dim3(kWave), 0, s, a);
  } else if (npl == 2) {
    hipLaunchKernelGGL(replay_kernel<2>, dim3(a.R), dim3(kWave), 0, s, a);
  } else {
    hipLaunchKernelGGL(replay_kernel<4>, dim3(a.R), dim3(kWave), 0, s, a);
  }
  return hipGetLastError();
}

hipError_t launch_rep_stats(const ReplayArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(rep_stats_kernel, dim3(a.R), dim3(kStatThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace fognet
