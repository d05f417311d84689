// replay_v2.hip — batched replay of FogNetSim++'s v2 offload model on gfx950
// (SURVEY.md §8(f) row 2): the modules simulations/example/wirelessNet.ini:56,62
// select,
//   broker  BrokerBaseApp2::handleMessageWhenUp/sendPubAck/releaseResource
//           BrokerBaseApp2.cc:62-203, 205-287, 382-406
//   node    ComputeBrokerApp2::advertiseMIPS/releaseResource/processPacket
//           ComputeBrokerApp2.cc:202-220, 222-245, 247-324
// The v2 model has periodic 10-ms node timers whose phase every accepted task
// resets, a broker timer that only local tasks re-arm, and double-valued
// deadlines whose rounding decides releases, so it is replayed as a
// discrete-event simulation in OMNeT++'s future-event order (tick, then
// insertion sequence) rather than in closed form.
//
// One wavefront replays one replication; node j lives on lane j (N <= 64):
// its remaining MIPS, the broker's advertised view of it, its self-message
// (tick, sequence, kind) and the heads of its two message queues in VGPRs
// (broker -> node tasks and node -> broker adverts/acks; latencies are fixed
// per node, so each queue is FIFO), the queue bodies and its reservation list
// in HBM.  Each step takes the earliest (tick, sequence) over the 64 lanes (two
// wave minima) and over the broker's own sources (the next trace publish,
// whose pre-insertion sequence is N + index, and the broker timer), then runs
// that one handler.  Broker state is wave-uniform; per-task outputs and the
// broker's request list are written by lane 0 only and a node's queues by its
// own lane only, so every memory location has one writer in program order.
#include <stdlib.h>
#include <string.h>

#include "replay_common.h"

namespace fognet {

namespace {

constexpr int64_t kAdvertPeriod = 10000000000LL;  // scheduleAt(simTime() + 0.01) (ComputeBrokerApp2.cc:219)
constexpr int64_t kMaxV2Tick = (int64_t)1 << 53;  // ticks convert to double exactly
constexpr uint32_t kKindAdvertise = 1u, kKindRelease = 2u;
constexpr int32_t kMsgAdvert = 1, kMsgAck6 = 2;
constexpr uint8_t kListNone = 0, kListLocal = 1, kListForwarded = 2;

// Adverts that change nothing.  A node's ADVERTISEMIPS firing (ComputeBrokerApp2.cc
// :202-220) sends its MIPS to the broker, whose handler only sets the node's view
// (BrokerBaseApp2.cc:128-136) and schedules nothing.  Adverts of one node travel
// one fixed-latency link, so they arrive in send order, and an advert carrying the
// same MIPS as the node's previous one finds that value in the view already: its
// arrival changes no state and inserts no event, so leaving it out of the queue
// changes neither the FES order nor any sequence number of the events that remain
// (its own insertion sequence is still consumed at the send).  Such an advert is
// only counted, as the event it is (`events`), if it arrives before the stop.  Per
// node at most one is in flight (a firing leaves it out only once the previous one
// has arrived; else it is queued like any other), so an error that ends the
// replication early un-counts at most that one.  At C1 these are the nodes'
// 10-ms adverts between two MIPS changes: about half of all FES events.
constexpr bool kPhantomAdverts = true;

// replay_v2_kernel<NPL>: from this many nodes per lane on, a node's state is split
// (the per-slot earliest event in VGPRs, the record indexed by slot; see the kernel)
#ifndef FOGNET_V2_COLD_NPL
#define FOGNET_V2_COLD_NPL 8
#endif

// Batched timer firings (replay_v2_rows_kernel).  A node's firing that releases
// nothing (ComputeBrokerApp2.cc:222-245 finds no expired reservation, or the
// self-message is ADVERTISEMIPS) touches only its node: it sends the advert
// (queued, or left out as above) and re-arms the self-message 0.01 s later,
// consuming two insertion sequence numbers.  The earliest firings of a row's
// nodes that precede every other pending event, the first firing that releases
// something and the arrival of any advert one of them queues are therefore the
// next events of the FES in their own (tick, sequence) order, and the rest of the
// simulation cannot observe that they are handled in one step: each takes the
// two sequence numbers its rank among them gives.  At C1 most events are such
// firings (five nodes, a 10-ms timer, a publish every 50 ms).
constexpr bool kBatchFirings = true;
// Periods per node in one rows-kernel batch (at most 3 * kBatchGens * 16 sequence
// numbers per 16-lane row and batch)
#ifndef FOGNET_V2_BATCH_GENS
#define FOGNET_V2_BATCH_GENS 5
#endif
constexpr int kBatchGens = FOGNET_V2_BATCH_GENS;
static_assert(kBatchGens >= 1 && kBatchGens <= 24, "release mask and the row broadcast's packing");
// The same batches in replay_v2_kernel<NPL> (N > 32), the firings ranked by a bitonic
// sort in LDS (FOGNET_V2_NPL_BATCH=0: one event per step, for A/B timing)
#ifndef FOGNET_V2_NPL_BATCH
#define FOGNET_V2_NPL_BATCH 1
#endif
constexpr bool kBatchNpl = FOGNET_V2_NPL_BATCH != 0;
constexpr int32_t kNoAdvert = INT32_MIN;  // no advert sent yet (the broker's view starts at MIPS 0)

struct V2Msg {  // a message in flight: arrival tick, insertion sequence, payload
  int64_t tick;
  uint64_t seq;
  int32_t kind;  // node -> broker: kMsgAdvert / kMsgAck6; broker -> node: the task's MIPSRequired
  int32_t val;   // task index, or the advertised MIPS
};

struct V2Res {  // a reservation at a node: Request{requiredTime = now.dbl() + requiredTime}
  int32_t task;
  int32_t req;  // its MIPSRequired
  double deadline;
};

// SimTime::dbl() of OMNeT++ 4.6: ticks times the double scale 1e-12.
__device__ __forceinline__ double dbl(int64_t t) { return mul_rn((double)t, 1e-12); }

// Wave minimum when only lanes < 16 can hold a candidate (N <= 16): the four
// in-row DPP butterflies of wave_min_u64, then row 0's value.
__device__ __forceinline__ uint64_t row0_min_u64(uint64_t v) {
  v = umin64(v, dpp_u64<0xB1>(v));
  v = umin64(v, dpp_u64<0x4E>(v));
  v = umin64(v, dpp_u64<0x141>(v));
  v = umin64(v, dpp_u64<0x140>(v));
  return (uint64_t)readlane_i64((int64_t)v, 0);
}

__device__ __forceinline__ bool earlier(int64_t t, uint64_t s, int64_t t2, uint64_t s2) {
  return t < t2 || (t == t2 && s < s2);
}

struct V2Args {
  fognet_v2_in in;
  fognet_v2_out out;
  V2Msg* inq;     // [R][64][Q]
  V2Msg* outq;    // [R][64][Q]
  V2Res* res;     // [R][64][Q]
  uint8_t* list;  // [R][T] broker request list membership (kList*)
  int32_t q_log2;
};

// Per-node state of replay_v2_kernel (node j = slot * 64 + lane).
struct V2Node {
  int32_t mips, view;  // remaining MIPS; the broker's view of it (starts at MIPS 0, BrokerBaseApp2.cc:105)
  int64_t dl, ul;
  bool t_sched;        // selfMsg->isScheduled()
  int64_t t_tick;
  uint64_t t_seq;
  uint32_t t_kind;
  uint32_t in_h, in_n, out_h, out_n, rs_h, rs_n;
  V2Msg in_hd, out_hd;
  // adverts that change nothing at the broker (kPhantomAdverts): the MIPS of the
  // node's last advert sent, its one unqueued advert in flight and the count of those
  int32_t last_sent;
  int64_t ph_tick;  // (INT64_MIN: none in flight)
  uint64_t ph_seq;
  uint32_t ph_cnt;
};

// NPL nodes per lane (N <= 64 * NPL): node j on lane j % 64, slot j / 64, like
// the v3 register kernel.  The slot is a compile-time index everywhere (static
// loops select it), so the state stays in registers.
// A lane's slots as a bit mask (bit s: slot s), one 64-bit word per 64 slots.
template <int W>
struct SlotBits {
  uint64_t w[W];
  __device__ __forceinline__ void set(int s) { w[s >> 6] |= 1ull << (s & 63); }
  __device__ __forceinline__ bool test(int s) const { return ((w[s >> 6] >> (s & 63)) & 1ull) != 0ull; }
  __device__ __forceinline__ uint32_t popc() const {
    uint32_t c = 0u;
#pragma unroll
    for (int i = 0; i < W; ++i) c += (uint32_t)__popcll(w[i]);
    return c;
  }
};

template <int NPL>
__global__ __launch_bounds__(64) void replay_v2_kernel(V2Args P) {
  constexpr int kPad = NPL * kWave;  // queue rows per replication
  const fognet_v2_in& A = P.in;
  const fognet_v2_out& O = P.out;
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = A.N, T = A.T;
  const uint32_t Q = 1u << P.q_log2, qm = Q - 1u;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  // queue row of slot s of this lane (node s * 64 + lane)
  auto qrow = [&](int s) -> size_t { return ((size_t)r * (size_t)kPad + (size_t)(s * kWave + lane)) << P.q_log2; };
  uint8_t* const list = P.list + tbase;
  const int64_t* const arrive = A.arrive_tick + tbase;
  const int32_t* const reqs = A.req_mips + tbase;

  const double rt = A.required_time_s[r];
  const double rtx = mul_rn(rt, 1e12);  // SimTime + double: the double in ticks
  const int64_t rt_ticks = (int64_t)add_rn(rtx, rtx >= 0.0 ? 0.5 : -0.5);
  const int64_t stop = A.stop_tick[r];

  V2Node nd[NPL];
  // NPL >= 8 (N > 256): a node's whole state does not fit in VGPRs next to the
  // others', so it is split.  Every step's scan reads, for every slot, the node's
  // earliest event (tick, sequence, source) and the broker's view of it: those stay
  // in VGPRs (static slot index); the rest of the node's state is touched only by
  // the handler of an event of that node (wave-uniform slot ws), so `nd` is indexed
  // by ws directly and goes to scratch, read by one handler per step instead of by
  // every step's scan.  NPL <= 4 keeps everything in VGPRs (static slot loops).
  constexpr bool kCold = NPL >= FOGNET_V2_COLD_NPL;
  using SlotMask = SlotBits<(NPL + 63) / 64>;
  int64_t h_tick[kCold ? NPL : 1];
  uint64_t h_seq[kCold ? NPL : 1];
  int32_t h_src[kCold ? NPL : 1], h_view[kCold ? NPL : 1];
  bool bad = !(stop <= kMaxV2Tick) || !(rtx >= 0.0) || rt_ticks > kMaxV2Tick;
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const int j = s * kWave + lane;
    V2Node& x = nd[s];
    x.mips = 0;
    x.view = 0;
    x.dl = x.ul = 0;
    x.t_sched = false;
    x.t_tick = kNever;
    x.t_seq = ~0ull;
    x.t_kind = kKindAdvertise;
    x.in_h = x.in_n = x.out_h = x.out_n = x.rs_h = x.rs_n = 0u;
    x.in_hd = V2Msg{kNever, ~0ull, 0, 0};
    x.out_hd = V2Msg{kNever, ~0ull, 0, 0};
    x.last_sent = kNoAdvert;
    x.ph_tick = INT64_MIN;
    x.ph_seq = 0ull;
    x.ph_cnt = 0u;
    if (j < N) {
      x.mips = A.mips[nbase + j];
      x.dl = A.dl_tick[nbase + j];
      x.ul = A.ul_tick[nbase + j];
      const int64_t fa = A.first_adv_tick[nbase + j];
      bad |= x.dl < 0 || x.ul < 0 || fa < 0 || x.dl > kMaxV2Tick || x.ul > kMaxV2Tick || fa > kMaxV2Tick;
      x.t_sched = true;  // the first ADVERTISEMIPS firing, pre-inserted in node order
      x.t_tick = fa;
      x.t_seq = (uint64_t)j;
    }
  }
  // a node's earliest event: its self-message, its next task arrival, its next message at the broker
  auto key_of = [](const V2Node& x, int64_t& kt, uint64_t& ks, int32_t& ksrc) {
    kt = kNever;
    ks = ~0ull;
    ksrc = 0;
    if (x.t_sched) {
      kt = x.t_tick;
      ks = x.t_seq;
      ksrc = 1;
    }
    if (x.in_n && earlier(x.in_hd.tick, x.in_hd.seq, kt, ks)) {
      kt = x.in_hd.tick;
      ks = x.in_hd.seq;
      ksrc = 2;
    }
    if (x.out_n && earlier(x.out_hd.tick, x.out_hd.seq, kt, ks)) {
      kt = x.out_hd.tick;
      ks = x.out_hd.seq;
      ksrc = 3;
    }
  };
  // refresh slot ws's VGPR copy from its record (kCold; the owner lane, after its handler)
  auto refresh = [&](int ws) {
    if constexpr (kCold) {
      int64_t kt;
      uint64_t ks;
      int32_t ksrc;
      const V2Node& x = nd[ws];
      key_of(x, kt, ks, ksrc);
      const int32_t v = x.view;
#pragma unroll
      for (int s2 = 0; s2 < NPL; ++s2) {
        if (s2 == ws) {
          h_tick[s2] = kt;
          h_seq[s2] = ks;
          h_src[s2] = ksrc;
          h_view[s2] = v;
        }
      }
    }
  };
  if constexpr (kCold) {
#pragma unroll
    for (int s = 0; s < NPL; ++s) {
      key_of(nd[s], h_tick[s], h_seq[s], h_src[s]);
      h_view[s] = nd[s].view;
    }
  }
  // the broker's view of slot s (this lane's node s * 64 + lane)
  auto view_of = [&](int s) -> int32_t {
    if constexpr (kCold) return h_view[s];
    else return nd[s].view;
  };
  // f(node, slot) over this lane's slots (all, or those of the bit mask m): a
  // counted loop over the scratch records (kCold; one copy of f), else unrolled
  // over the register-resident ones
  auto for_slots = [&](auto&& f) {
    if constexpr (kCold) {
#pragma unroll 1
      for (int s = 0; s < NPL; ++s) f(nd[s], s);
    } else {
#pragma unroll
      for (int s = 0; s < NPL; ++s) f(nd[s], s);
    }
  };
  auto for_slots_in = [&](const SlotMask& m, auto&& f) {
    if constexpr (kCold) {
#pragma unroll 1
      for (int i = 0; i < (NPL + 63) / 64; ++i) {
        for (uint64_t x = m.w[i]; x; x &= x - 1ull) {
          const int s = i * 64 + (int)__builtin_ctzll(x);
          f(nd[s], s);
        }
      }
    } else {
#pragma unroll
      for (int s = 0; s < NPL; ++s)
        if (m.test(s)) f(nd[s], s);
    }
  };
  // batch ranks (kBatchFirings): the batch's firings as (tick, seq << 15 | releases << 14 |
  // node) sorted in LDS; then each firing's sequence-number offset, by node (aliasing the
  // ticks, dead once sorted: 32-bit offsets while the sort holds a firing per node, 16-bit
  // above, where a batch is cut at kSortCap firings)
  constexpr int kSortCap = NPL * kWave <= 8192 ? NPL * kWave : 4096;
  using OffT = std::conditional_t<(kSortCap < NPL * kWave), uint16_t, uint32_t>;
  __shared__ int64_t s_bt[kSortCap];
  __shared__ uint64_t s_bk[kSortCap];
  OffT* const s_off = reinterpret_cast<OffT*>(s_bt);
  static_assert(NPL * kWave <= (1 << 14), "node index in 14 bits of the batch key");
  static_assert(sizeof(OffT) * NPL * kWave <= sizeof(int64_t) * kSortCap, "offsets alias the sorted ticks");
  static_assert(sizeof(OffT) == 4 || 3 * kSortCap < 65536, "16-bit offsets: 2 i + releases < 3 kSortCap");

  // ---- broker (wave-uniform)
  int32_t pool = A.broker_mips[r];
  bool b_sched = false;
  int64_t b_tick = kNever;
  uint64_t b_seq = ~0ull;
  uint64_t seq = (uint64_t)N + (uint64_t)T;  // the publishes hold N .. N+T-1
  int next = 0, list_h = 0;
  int64_t prev_pub = INT64_MIN;
  // the next publish, loaded one publish ahead
  int64_t p_tick = T > 0 ? arrive[0] : kNever;
  int32_t p_req = T > 0 ? reqs[0] : 0;
  fognet_v2_stats st = {};
  uint32_t err = ballot(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;
  bad = false;
  int64_t end_tick = kNever;  // the last event dispatched (where an error ends the replication)
  uint64_t end_seq = ~0ull;

  while (err == FOGNET_OK) {
    // ---- the earliest event: the lanes' own sources (over their slots), then the broker's
    int64_t ct = kNever;
    uint64_t cs = ~0ull;
    int src = 0;  // 1 self-message, 2 task arrival, 3 message at the broker
    int csl = 0;  // its slot
#pragma unroll
    for (int s = 0; s < NPL; ++s) {
      if constexpr (kCold) {
        if (h_src[s] && earlier(h_tick[s], h_seq[s], ct, cs)) {
          ct = h_tick[s];
          cs = h_seq[s];
          src = h_src[s];
          csl = s;
        }
      } else {
        const V2Node& x = nd[s];
        if (x.t_sched && earlier(x.t_tick, x.t_seq, ct, cs)) {
          ct = x.t_tick;
          cs = x.t_seq;
          src = 1;
          csl = s;
        }
        if (x.in_n && earlier(x.in_hd.tick, x.in_hd.seq, ct, cs)) {
          ct = x.in_hd.tick;
          cs = x.in_hd.seq;
          src = 2;
          csl = s;
        }
        if (x.out_n && earlier(x.out_hd.tick, x.out_hd.seq, ct, cs)) {
          ct = x.out_hd.tick;
          cs = x.out_hd.seq;
          src = 3;
          csl = s;
        }
      }
    }
    const int64_t m_tick =
        (int64_t)((NPL == 1 && N <= 16) ? row0_min_u64((uint64_t)ct) : wave_min_u64((uint64_t)ct));
    const uint64_t tied = ballot(src != 0 && ct == m_tick);
    uint64_t m_seq = ~0ull, wmask = tied;
    if (__popcll(tied) > 1) {  // same-tick events on several lanes: insertion order decides
      m_seq = (NPL == 1 && N <= 16) ? row0_min_u64(ct == m_tick ? cs : ~0ull)
                                    : wave_min_u64(ct == m_tick ? cs : ~0ull);
      wmask = ballot(src != 0 && ct == m_tick && cs == m_seq);
    } else if (tied) {
      m_seq = ((uint64_t)readlane_u32((uint32_t)(cs >> 32), __builtin_ctzll(tied)) << 32) |
              readlane_u32((uint32_t)cs, __builtin_ctzll(tied));
    }
    const int w = wmask ? (int)__builtin_ctzll(wmask) : 0;
    int kind = wmask ? 1 : 0;  // 1 node-side event of lane w, 2 publish, 3 broker timer
    int64_t e_tick = wmask ? m_tick : kNever;
    uint64_t e_seq = wmask ? m_seq : ~0ull;
    if (next < T) {
      if (earlier(p_tick, (uint64_t)N + (uint64_t)next, e_tick, e_seq)) {
        e_tick = p_tick;
        e_seq = (uint64_t)N + (uint64_t)next;
        kind = 2;
      }
    }
    if (b_sched && earlier(b_tick, b_seq, e_tick, e_seq)) {
      e_tick = b_tick;
      e_seq = b_seq;
      kind = 3;
    }
    if (kind == 0 || e_tick >= stop) break;  // nothing left, or the sim-time-limit

    // ---- a batch (kBatchFirings, the rows kernel's rule over NPL nodes per lane).  When
    // the earliest event is a node's timer firing or a message reaching the broker, every
    // node's next firing and every node -> broker message before H -- the earliest task
    // arrival, publish or broker RELEASERESOURCE: the events that draw sequence numbers
    // and touch a node or the request list -- are handled in this one step.  A firing
    // touches only its node and draws two sequence numbers (three when it releases a
    // reservation: its status-6 ack's first), a message draws none and touches only the
    // broker's view or, for an ack, its request's list entry, so they commute; each
    // firing takes the numbers its (tick, sequence) rank among the batch's firings gives
    // (a bitonic sort of the batch in LDS), and each node's messages are popped in its
    // FIFO's order (its own firing's advert included when it lands before H).
    if (kBatchNpl && kind == 1 && (int)readlane_u32((uint32_t)src, w) != 2) {
      int64_t ht = kNever;
      uint64_t hs = ~0ull;
      for_slots([&](V2Node& x, int) {
        if (x.in_n && earlier(x.in_hd.tick, x.in_hd.seq, ht, hs)) {
          ht = x.in_hd.tick;
          hs = x.in_hd.seq;
        }
      });
      int64_t H_t = (int64_t)wave_min_u64((uint64_t)ht);
      uint64_t H_s = wave_min_u64(ht == H_t ? hs : ~0ull);
      if (next < T && earlier(p_tick, (uint64_t)N + (uint64_t)next, H_t, H_s)) {
        H_t = p_tick;
        H_s = (uint64_t)N + (uint64_t)next;
      }
      if (b_sched && earlier(b_tick, b_seq, H_t, H_s)) {
        H_t = b_tick;
        H_s = b_seq;
      }
      // the batch's firings (bit s: slot s), and those that release a reservation
      // (ComputeBrokerApp2.cc:222-226: the oldest, when its deadline < now)
      SlotMask cm{}, rm{};
      for_slots([&](V2Node& x, int s) {
        if (x.t_sched && x.t_tick < stop && earlier(x.t_tick, x.t_seq, H_t, H_s)) {
          cm.set(s);
          if (x.t_kind == kKindRelease && x.rs_n) {
            const V2Res h = P.res[qrow(s) + (x.rs_h & qm)];
            if (h.deadline < dbl(x.t_tick)) rm.set(s);
          }
        }
      });
      uint32_t c = cm.popc();
      uint32_t c_incl = wave_scan_add_u32(c);
      uint32_t n = readlane_u32(c_incl, kWave - 1);
      if constexpr (kSortCap < NPL * kWave) {
        if (n > (uint32_t)kSortCap) {
          // more firings than the LDS sort holds: the batch ends earlier, at the largest (tick,
          // seq) bound H' with at most kSortCap firings before it (binary searches over the
          // tick, then the sequence at that tick); the events from H' on are the next step's.
          // At least the current event (a firing at e_tick, e_seq) stays before it.
          auto before = [&](int64_t bt, uint64_t bs) -> uint32_t {
            uint32_t k = 0u;
            for_slots_in(cm, [&](V2Node& x, int) { k += earlier(x.t_tick, x.t_seq, bt, bs) ? 1u : 0u; });
            return wave_sum_u32(k);
          };
          // before(lo, 0) == 0; before(hi, 0) >= n > cap (every firing of the batch is before stop)
          int64_t lo = e_tick, hi = H_t < stop ? H_t + 1 : stop;
          while (hi - lo > 1) {
            const int64_t mid = lo + (hi - lo) / 2;
            if (before(mid, 0ull) <= (uint32_t)kSortCap) lo = mid;
            else hi = mid;
          }
          uint64_t slo = 0ull, shi = ~0ull;  // at tick lo: before(lo, ~0) covers every firing at lo
          while (shi - slo > 1ull) {
            const uint64_t mid = slo + (shi - slo) / 2ull;
            if (before(lo, mid) <= (uint32_t)kSortCap) slo = mid;
            else shi = mid;
          }
          H_t = lo;
          H_s = slo;
          SlotMask cm2{}, rm2{};
          for_slots_in(cm, [&](V2Node& x, int s) {
            if (earlier(x.t_tick, x.t_seq, H_t, H_s)) {
              cm2.set(s);
              if (rm.test(s)) rm2.set(s);
            }
          });
          cm = cm2;
          rm = rm2;
          c = cm.popc();
          c_incl = wave_scan_add_u32(c);
          n = readlane_u32(c_incl, kWave - 1);
        }
      }
      if (seq >= (1ull << 48)) {  // (the sort key keeps the sequence in 49 bits)
        err = FOGNET_ERR_CAPACITY;
        break;
      }
      uint32_t p = c_incl - c;
      for_slots_in(cm, [&](V2Node& x, int s) {
        s_bt[p] = x.t_tick;
        s_bk[p] = (x.t_seq << 15) | ((uint64_t)(rm.test(s) ? 1u : 0u) << 14) | (uint64_t)(s * kWave + lane);
        ++p;
      });
      uint32_t n2 = 1u;
      while (n2 < n) n2 <<= 1;
      for (uint32_t i = n + (uint32_t)lane; i < n2; i += kWave) {
        s_bt[i] = INT64_MAX;
        s_bk[i] = ~0ull;
      }
      __syncthreads();
      for (uint32_t k = 2u; k <= n2; k <<= 1) {
        for (uint32_t j = k >> 1; j > 0u; j >>= 1) {
          for (uint32_t i = (uint32_t)lane; i < n2; i += kWave) {
            const uint32_t q = i ^ j;
            if (q > i) {
              const int64_t ti = s_bt[i], tq = s_bt[q];
              const uint64_t ki = s_bk[i], kq = s_bk[q];
              const bool gt = ti > tq || (ti == tq && ki > kq);
              if (gt == ((i & k) == 0u)) {
                s_bt[i] = tq;
                s_bt[q] = ti;
                s_bk[i] = kq;
                s_bk[q] = ki;
              }
            }
          }
          __syncthreads();
        }
      }
      // sorted position i draws from seq + 2 i + (releasing firings before it)
      uint32_t n_relb = 0u;
      for (uint32_t b0 = 0u; b0 < n; b0 += kWave) {
        const uint32_t i = b0 + (uint32_t)lane;
        const uint64_t kx = i < n ? s_bk[i] : 0ull;
        const uint32_t rl = i < n ? (uint32_t)(kx >> 14) & 1u : 0u;
        const uint32_t incl = wave_scan_add_u32(rl);
        if (i < n) s_off[kx & 0x3FFFu] = (OffT)(2u * i + n_relb + incl - rl);
        n_relb += readlane_u32(incl, kWave - 1);
      }
      __syncthreads();
      const uint32_t tot = 2u * n + n_relb;
      uint32_t n_rel = 0u;
      bool has_last = false;
      int64_t lt_t = 0;
      uint64_t lt_s = 0ull;
      for_slots_in(cm, [&](V2Node& x, int s) {
        const uint32_t off = s_off[s * kWave + lane];
        const bool rel = rm.test(s);
        uint64_t sq = seq + off;
        const int64_t ft = x.t_tick;
        const uint64_t fs = x.t_seq;
        V2Msg* const outq = P.outq + qrow(s);
        auto push_out = [&](const V2Msg& m) {
          if (x.out_n == Q) {
            bad = true;
          } else {
            outq[(x.out_h + x.out_n) & qm] = m;
            if (x.out_n == 0u) x.out_hd = m;
            ++x.out_n;
          }
        };
        if (rel) {  // releaseResource: the oldest reservation, acked with status 6 (:225-235)
          const V2Res h = P.res[qrow(s) + (x.rs_h & qm)];
          x.mips += h.req;  // :226
          ++x.rs_h;
          --x.rs_n;
          O.done_tick[tbase + h.task] = ft;
          ++n_rel;
          push_out(V2Msg{ft + x.ul, sq++, kMsgAck6, h.task});
        }
        // advertiseMIPS (:202-220): advert, then the self-message again 0.01 s later
        if (kPhantomAdverts && x.mips == x.last_sent && earlier(x.ph_tick, x.ph_seq, ft, fs)) {
          x.ph_tick = ft + x.ul;
          x.ph_seq = sq++;
          x.ph_cnt += x.ph_tick < stop ? 1u : 0u;
        } else {
          push_out(V2Msg{ft + x.ul, sq++, kMsgAdvert, x.mips});
          x.last_sent = x.mips;
        }
        x.t_sched = true;
        x.t_tick = ft + kAdvertPeriod;
        x.t_seq = sq++;
        if (off + (rel ? 3u : 2u) == tot) {  // the batch's last firing
          has_last = true;
          lt_t = ft;
          lt_s = fs;
        }
      });
      // node -> broker messages before H (BrokerBaseApp2.cc:128-154), per node in FIFO order
      uint32_t n_arr = 0u, n_rl = 0u;
      for_slots([&](V2Node& x, int s) {
        while (x.out_n && x.out_hd.tick < stop && earlier(x.out_hd.tick, x.out_hd.seq, H_t, H_s)) {
          if (x.out_hd.kind == kMsgAdvert) {
            x.view = x.out_hd.val;  // setMips (:132)
          } else if (list[x.out_hd.val] == kListForwarded) {  // ack 6: relay, erase if still listed
            list[x.out_hd.val] = kListNone;
            ++n_rl;
          }
          ++x.out_h;
          --x.out_n;
          if (x.out_n) x.out_hd = P.outq[qrow(s) + (x.out_h & qm)];
          ++n_arr;
        }
      });
      if constexpr (kCold) {
#pragma unroll
        for (int s = 0; s < NPL; ++s) {
          key_of(nd[s], h_tick[s], h_seq[s], h_src[s]);
          h_view[s] = nd[s].view;
        }
      }
      st.events += (int64_t)n + (int64_t)wave_sum_u32(n_arr);
      st.n_released_node += (int64_t)wave_sum_u32(n_rel);
      st.n_relayed += (int64_t)wave_sum_u32(n_rl);
      seq += tot;
      if (n) {  // where an error ends the replication: the batch's last firing
        const int wl = (int)__builtin_ctzll(ballot(has_last));
        end_tick = readlane_i64(lt_t, wl);
        end_seq = (uint64_t)readlane_i64((int64_t)lt_s, wl);
      }
      if (ballot(bad)) {
        err = FOGNET_ERR_CAPACITY;
        break;
      }
      continue;
    }

    const int64_t now = e_tick;
    ++st.events;
    end_tick = e_tick;
    end_seq = e_seq;

    if (kind == 2) {
      // ---- publish: BrokerBaseApp2.cc:176-195 + sendPubAck(:205-287)
      const int t = next++;
      if (p_tick < prev_pub || p_tick > kMaxV2Tick) {
        err = FOGNET_ERR_ARG;  // trace not sorted / out of range
        break;
      }
      prev_pub = p_tick;
      const int32_t req = p_req;
      if (next < T) {  // the following publish, in flight while this one is handled
        p_tick = arrive[next];
        p_req = reqs[next];
      }
      ++st.n_tasks;
      int32_t k = -1;
      uint32_t status;
      int64_t start = -1;
      uint8_t lmark = kListNone;
      if (req < pool) {  // :181 -> sendPubAck(true), :209-232
        pool -= req;
        lmark = kListLocal;
        status = FOGNET_V2_ST_LOCAL;
        start = now;
        ++st.n_local;
        b_sched = true;  // cancelEvent + scheduleAt(now + requiredTime) (:226-229)
        b_tick = now + rt_ticks;
        b_seq = seq++;
      } else if (N == 0) {  // :273-285: scheduleAt without cancelEvent
        status = FOGNET_V2_ST_NO_NODES;
        ++st.n_no_nodes;
        if (b_sched) {
          err = FOGNET_ERR_STATE;  // "scheduleAt(): message already scheduled"
        } else {
          b_sched = true;
          b_tick = now + rt_ticks;
          b_seq = seq++;
        }
      } else {
        // the LAST node whose advertised MIPS exceeds node 0's (:241-248), else node 0
        const int32_t v0 = (int32_t)readlane_u32((uint32_t)view_of(0), 0);
        uint32_t last = 0u;
#pragma unroll
        for (int s = 0; s < NPL; ++s) {
          const int j = s * kWave + lane;
          if (j < N && j >= 1 && view_of(s) > v0) last = (uint32_t)j;
        }
        k = (int32_t)~wave_min_u32(~last);
        const int kl = k & (kWave - 1), ks = k / kWave;
        int32_t vk = 0;
#pragma unroll
        for (int s = 0; s < NPL; ++s)
          if (s == ks) vk = (int32_t)readlane_u32((uint32_t)view_of(s), kl);
        lmark = kListForwarded;  // :255-260, before the MIPS check
        if (req < vk) {          // :262-270: FognetMsgTask to node k
          status = FOGNET_V2_ST_FORWARDED;
          ++st.n_forwarded;
          if (lane == kl) {
            auto push = [&](V2Node& x, int s) {
              const V2Msg m = {now + x.dl, seq, req, t};
              if (x.in_n == Q) {
                bad = true;
              } else {
                P.inq[qrow(s) + ((x.in_h + x.in_n) & qm)] = m;
                if (x.in_n == 0u) x.in_hd = m;
                ++x.in_n;
              }
            };
            if constexpr (kCold) {
              push(nd[ks], ks);
              refresh(ks);
            } else {
#pragma unroll
              for (int s = 0; s < NPL; ++s)
                if (s == ks) push(nd[s], s);
            }
          }
          ++seq;
          if (ballot(bad)) err = FOGNET_ERR_CAPACITY;
        } else {
          status = FOGNET_V2_ST_DROPPED;
          ++st.n_dropped;
        }
      }
      if (lane == 0) {
        list[t] = lmark;
        O.node[tbase + t] = k;
        O.status[tbase + t] = (uint8_t)status;
        O.start_tick[tbase + t] = start;
        O.done_tick[tbase + t] = -1;
      }
    } else if (kind == 3) {
      // ---- broker RELEASERESOURCE: BrokerBaseApp2::releaseResource (:382-406), the
      // first request with deadline <= now (the oldest live one: deadlines follow
      // the list order), local or forwarded
      b_sched = false;
      int rel = -1;
      uint32_t mark = kListNone;
      if (lane == 0) {
        while (list_h < next && list[list_h] == kListNone) ++list_h;
        if (list_h < next) {
          const double deadline = add_rn(dbl(arrive[list_h]), rt);
          if (deadline <= dbl(now)) {
            rel = list_h;
            mark = list[list_h];
            list[list_h] = kListNone;
            if (mark == kListLocal) O.done_tick[tbase + list_h] = now;
          }
        }
      }
      list_h = __builtin_amdgcn_readfirstlane(list_h);
      rel = __builtin_amdgcn_readfirstlane(rel);
      mark = __builtin_amdgcn_readfirstlane(mark);
      if (rel >= 0) {
        pool += reqs[rel];  // :386
        ++st.n_released_broker;
        if (mark == kListForwarded) ++st.n_inflated;
      }
    } else {
      // ---- an event of node ws * 64 + w
      const int wsrc = (int)readlane_u32((uint32_t)src, w);
      const int ws = (int)readlane_u32((uint32_t)csl, w);
      if (wsrc == 3) {
        // a node -> broker message reaches the broker (BrokerBaseApp2.cc:128-154)
        int32_t mk = 0, mv = 0;
        auto receive = [&](V2Node& x, int s) {
          mk = (int32_t)readlane_u32((uint32_t)x.out_hd.kind, w);
          mv = (int32_t)readlane_u32((uint32_t)x.out_hd.val, w);
          if (lane == w) {
            ++x.out_h;
            --x.out_n;
            if (x.out_n) x.out_hd = P.outq[qrow(s) + (x.out_h & qm)];
            if (mk == kMsgAdvert) x.view = mv;  // setMips (:132)
          }
        };
        if constexpr (kCold) {
          receive(nd[ws], ws);
          if (lane == w) refresh(ws);
        } else {
#pragma unroll
          for (int s = 0; s < NPL; ++s)
            if (s == ws) receive(nd[s], s);
        }
        if (mk == kMsgAck6) {  // relay and erase the request if it is still listed (:145-153)
          bool relayed = false;
          if (lane == 0 && list[mv] == kListForwarded) {
            list[mv] = kListNone;
            relayed = true;
          }
          if (ballot(relayed)) ++st.n_relayed;
        }
      } else {
        // the node's own events: its self-message or a task arrival.  The owner
        // lane runs the handler; sequence numbers and per-task results are
        // broadcast afterwards (lane 0 writes the outputs).
        int32_t o_task = -1;   // task whose result changed
        uint32_t o_what = 0u;  // 1 released, 2 accepted, 3 rejected
        uint64_t my_seq = seq;
        auto handle = [&](V2Node& x, int s) {
            V2Msg* const outq = P.outq + qrow(s);
            if (wsrc == 1) {
              x.t_sched = false;
              if (x.t_kind == kKindRelease && x.rs_n) {
                // ComputeBrokerApp2::releaseResource (:222-245): the first reservation
                // with deadline < now (the oldest: deadlines follow arrival order)
                const V2Res h = P.res[qrow(s) + (x.rs_h & qm)];
                if (h.deadline < dbl(now)) {
                  x.mips += h.req;  // :226
                  ++x.rs_h;
                  --x.rs_n;
                  o_task = h.task;
                  o_what = 1u;
                  const V2Msg m = {now + x.ul, my_seq++, kMsgAck6, h.task};  // puback 6 (:231-235)
                  if (x.out_n == Q) bad = true;
                  else {
                    outq[(x.out_h + x.out_n) & qm] = m;
                    if (x.out_n == 0u) x.out_hd = m;
                    ++x.out_n;
                  }
                }
              }
              // advertiseMIPS (:202-220): advert, then the self-message again 0.01 s later
              if (kPhantomAdverts && x.mips == x.last_sent && earlier(x.ph_tick, x.ph_seq, now, e_seq)) {
                // carries the value of the node's previous advert, which the broker already holds
                x.ph_tick = now + x.ul;
                x.ph_seq = my_seq++;
                x.ph_cnt += x.ph_tick < stop ? 1u : 0u;
              } else {
                const V2Msg m = {now + x.ul, my_seq++, kMsgAdvert, x.mips};
                x.last_sent = x.mips;
                if (x.out_n == Q) bad = true;
                else {
                  outq[(x.out_h + x.out_n) & qm] = m;
                  if (x.out_n == 0u) x.out_hd = m;
                  ++x.out_n;
                }
              }
              x.t_sched = true;
              x.t_tick = now + kAdvertPeriod;
              x.t_seq = my_seq++;
            } else {
              // ComputeBrokerApp2::processPacket, FognetMsgTask (:258-318)
              const int32_t t = x.in_hd.val;
              const int32_t req = x.in_hd.kind;
              ++x.in_h;
              --x.in_n;
              if (x.in_n) x.in_hd = P.inq[qrow(s) + (x.in_h & qm)];
              o_task = t;
              if (req < x.mips) {  // :269
                x.mips -= req;     // :272
                o_what = 2u;
                if (x.rs_n == Q) bad = true;
                else {
                  P.res[qrow(s) + ((x.rs_h + x.rs_n) & qm)] = V2Res{t, req, add_rn(dbl(now), rt)};  // :274
                  ++x.rs_n;
                }
                // cancelEvent + RELEASERESOURCE at now + requiredTime (:292-295)
                x.t_kind = kKindRelease;
                x.t_sched = true;
                x.t_tick = now + rt_ticks;
                x.t_seq = my_seq++;
              } else {
                o_what = 3u;  // TaskAck(false) (:299-306)
              }
            }
        };
        if (lane == w) {
          if constexpr (kCold) {
            handle(nd[ws], ws);
            refresh(ws);
          } else {
#pragma unroll
            for (int s = 0; s < NPL; ++s)
              if (s == ws) handle(nd[s], s);
          }
        }
        if (ballot(bad)) {
          err = FOGNET_ERR_CAPACITY;
          break;
        }
        seq = ((uint64_t)readlane_u32((uint32_t)(my_seq >> 32), w) << 32) | readlane_u32((uint32_t)my_seq, w);
        o_task = (int32_t)readlane_u32((uint32_t)o_task, w);
        o_what = readlane_u32(o_what, w);
        if (o_what == 1u) {
          ++st.n_released_node;
          if (lane == 0) O.done_tick[tbase + o_task] = now;
        } else if (o_what == 2u) {
          ++st.n_accepted;
          if (lane == 0) {
            O.status[tbase + o_task] = FOGNET_V2_ST_ACCEPTED;
            O.start_tick[tbase + o_task] = now;
          }
        } else if (o_what == 3u) {
          ++st.n_rejected;
          if (lane == 0) O.status[tbase + o_task] = FOGNET_V2_ST_REJECTED;
        }
      }
    }
  }

  // ---- unqueued adverts dispatched before the end (an error ends the replication at
  // event end_*: the one still in flight after it is not)
  int64_t ph_sum = 0, msum = 0;
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    V2Node& x = nd[s];
    if (err != FOGNET_OK && x.ph_tick < stop && !earlier(x.ph_tick, x.ph_seq, end_tick, end_seq)) x.ph_cnt -= 1u;
    ph_sum += (int64_t)x.ph_cnt;
    msum += s * kWave + lane < N ? (int64_t)x.mips : 0;
  }
  for (int m = kWave / 2; m > 0; m >>= 1) ph_sum += (int64_t)shfl_xor_u64((uint64_t)ph_sum, m);
  st.events += ph_sum;
  // ---- tasks not published before the stop (or the error), and the record
  for (int t = next + lane; t < T; t += kWave) {
    O.node[tbase + t] = -1;
    O.status[tbase + t] = 0;
    O.start_tick[tbase + t] = -1;
    O.done_tick[tbase + t] = -1;
  }
  for (int m = kWave / 2; m > 0; m >>= 1) msum += (int64_t)shfl_xor_u64((uint64_t)msum, m);
  if (lane == 0) {
    st.node_mips_final_sum = msum;
    st.broker_mips_final = pool;
    st.status = (int32_t)err;
    O.stats[r] = st;
  }
}

// ---- four replications per wavefront (N <= 16): replication 4 * blockIdx.x + q
// on the 16-lane DPP row q = lane / 16, node j on lane 16 q + j.  The v2 loop is
// VALU-issue-bound (round 2: VALU busy 0.87 at 5 of 64 lanes holding nodes), so
// packing four replications into the lanes the one-per-wave kernel leaves idle
// runs four event loops per instruction stream.  Broker state that
// replay_v2_kernel keeps wave-uniform is row-uniform here (every lane of a row
// holds the same value); the earliest event is a row minimum (the four in-row
// DPP butterflies leave it in every lane of the row), a node's values reach the
// rest of its row with ds_bpermute, and every handler runs under a row-uniform
// condition, so rows in different handlers only serialise those handlers.
// Same arithmetic, same FES order, same outputs as replay_v2_kernel.
// Row width W (16 or 32 lanes): W = 16 packs four replications per wavefront
// (1,024 waves at the C1 size, one per SIMD); W = 32 packs two (2,048 waves, two
// per SIMD, so one wave's latencies overlap the other's work).
template <int W>
__device__ __forceinline__ uint64_t row_min_u64(uint64_t v) {
  v = umin64(v, dpp_u64<0xB1>(v));
  v = umin64(v, dpp_u64<0x4E>(v));
  v = umin64(v, dpp_u64<0x141>(v));
  v = umin64(v, dpp_u64<0x140>(v));
  if constexpr (W == 32) v = umin64(v, shfl_xor_u64(v, 16));
  return v;
}

template <int W>
__device__ __forceinline__ uint32_t row_min_u32(uint32_t v) {
  v = min(v, dpp_u32<0xB1>(v));
  v = min(v, dpp_u32<0x4E>(v));
  v = min(v, dpp_u32<0x141>(v));
  v = min(v, dpp_u32<0x140>(v));
  if constexpr (W == 32) v = min(v, (uint32_t)__shfl_xor((int)v, 16, kWave));
  return v;
}

template <int W>
__device__ __forceinline__ int64_t row_sum_i64(int64_t v) {
  v += (int64_t)dpp_u64<0xB1>((uint64_t)v);
  v += (int64_t)dpp_u64<0x4E>((uint64_t)v);
  v += (int64_t)dpp_u64<0x141>((uint64_t)v);
  v += (int64_t)dpp_u64<0x140>((uint64_t)v);
  if constexpr (W == 32) v += (int64_t)shfl_xor_u64((uint64_t)v, 16);
  return v;
}

// value of lane w of this lane's row (every lane of the row active)
template <int W>
__device__ __forceinline__ uint32_t row_bcast_u32(uint32_t v, int w) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((threadIdx.x & ~(W - 1u)) | (uint32_t)w) << 2), (int)v);
}

template <int W>
__device__ __forceinline__ uint64_t row_bcast_u64(uint64_t v, int w) {
  return ((uint64_t)row_bcast_u32<W>((uint32_t)(v >> 32), w) << 32) | row_bcast_u32<W>((uint32_t)v, w);
}

// some lane of this lane's row has p (the row's lanes active)
template <int W>
__device__ __forceinline__ bool row_any(bool p) {
  return ((ballot(p) >> (threadIdx.x & ~(W - 1u))) & ((1ull << W) - 1ull)) != 0ull;
}

// The rows kernel's queue entry: V2Msg with a 32-bit insertion sequence (the
// same 24-B slot of the workspace).  Sequence numbers start at N + T and grow
// by at most three per event; a replication that would pass 2^32 - 256 is
// refused (FOGNET_ERR_CAPACITY), so they never wrap.
struct V2MsgR {
  int64_t tick;
  uint32_t seq;
  int32_t kind;
  int32_t val;
  int32_t pad;
};
static_assert(sizeof(V2MsgR) == sizeof(V2Msg), "same queue slot");
constexpr uint32_t kSeqLimit = 0xFFFFFF00u;

constexpr int kTraceChunk = 64;

__device__ __forceinline__ bool earlier32(int64_t t, uint32_t s, int64_t t2, uint32_t s2) {
  return t < t2 || (t == t2 && s < s2);
}

template <int kRowLanes, int kActive = kWave / kRowLanes>
__global__ __launch_bounds__(64) void replay_v2_rows_kernel(V2Args P) {
  constexpr int kRowsPerWave = kWave / kRowLanes;
  const fognet_v2_in& A = P.in;
  const fognet_v2_out& O = P.out;
  const int lane = threadIdx.x;
  const int li = lane & (kRowLanes - 1);
  // (kActive < kRowsPerWave: only the first kActive rows replay, the others idle -- more
  // wavefronts, each issuing the union of fewer rows' paths)
  const int r = blockIdx.x * kActive + lane / kRowLanes;
  const bool live = lane / kRowLanes < kActive && r < A.R;  // rows past R idle from the start
  const int rr = live ? r : 0;  // (their addresses stay in bounds)
  const int N = A.N, T = A.T;
  const bool own = live && li < N;
  const uint32_t Q = 1u << P.q_log2, qm = Q - 1u;
  const size_t nbase = (size_t)rr * (size_t)A.node_stride;
  const size_t tbase = (size_t)rr * (size_t)T;
  const size_t qbase = ((size_t)rr * (size_t)kWave + (size_t)li) << P.q_log2;
  V2MsgR* const inq = reinterpret_cast<V2MsgR*>(P.inq) + qbase;
  V2MsgR* const outq = reinterpret_cast<V2MsgR*>(P.outq) + qbase;
  V2Res* const res = P.res + qbase;
  uint8_t* const list = P.list + tbase;
  const int64_t* const arrive = A.arrive_tick + tbase;
  const int32_t* const reqs = A.req_mips + tbase;

  const double rt = A.required_time_s[rr];
  const double rtx = mul_rn(rt, 1e12);  // SimTime + double: the double in ticks
  const int64_t rt_ticks = (int64_t)add_rn(rtx, rtx >= 0.0 ? 0.5 : -0.5);
  const int64_t stop = A.stop_tick[rr];

  // ---- node li of the row's replication
  int32_t mips = 0, view = 0;  // the broker's Broker record starts at MIPS 0 (BrokerBaseApp2.cc:105)
  int64_t dl = 0, ul = 0;
  bool t_sched = false;  // selfMsg->isScheduled()
  int64_t t_tick = kNever;
  uint32_t t_seq = ~0u;
  uint32_t t_kind = kKindAdvertise;
  bool bad = !(stop <= kMaxV2Tick) || !(rtx >= 0.0) || rt_ticks > kMaxV2Tick;
  if (own) {
    mips = A.mips[nbase + li];
    dl = A.dl_tick[nbase + li];
    ul = A.ul_tick[nbase + li];
    const int64_t fa = A.first_adv_tick[nbase + li];
    bad |= dl < 0 || ul < 0 || fa < 0 || dl > kMaxV2Tick || ul > kMaxV2Tick || fa > kMaxV2Tick;
    t_sched = true;  // the first ADVERTISEMIPS firing, pre-inserted in node order
    t_tick = fa;
    t_seq = (uint32_t)li;
  }
  // The node's three FIFOs (broker -> node tasks, node -> broker messages,
  // reservations) keep their first two entries in registers (hd, nx) and only the
  // rest in HBM: a push stores only from the third entry on, and a pop loads (and
  // waits for, sync_vm) only when a third entry moves up.  No load is then left in
  // flight across loop iterations: the compiler would wait for it at its first use
  // in a later step with vmcnt(0), which on gfx9 also waits for every store issued
  // since (the per-task outputs), i.e. an HBM write round trip per step.
  uint32_t in_h = 0u, in_n = 0u, out_h = 0u, out_n = 0u, rs_h = 0u, rs_n = 0u;
  V2MsgR in_hd = {kNever, ~0u, 0, 0, 0}, out_hd = {kNever, ~0u, 0, 0, 0};
  V2MsgR in_nx = in_hd, out_nx = out_hd;
  V2Res rs_hd = {0, 0, 0.0}, rs_nx = rs_hd;
  // unqueued adverts (kPhantomAdverts)
  int32_t last_sent = kNoAdvert;
  int64_t ph_tick = INT64_MIN;  // (none in flight)
  uint32_t ph_seq = 0u, ph_cnt = 0u;

  // ---- broker (row-uniform)
  int32_t pool = live ? A.broker_mips[rr] : 0;
  bool b_sched = false;
  int64_t b_tick = kNever;
  uint32_t b_seq = ~0u;
  uint32_t seq = (uint32_t)N + (uint32_t)T;  // the publishes hold N .. N+T-1
  int next = 0, list_h = 0;
  int64_t prev_pub = INT64_MIN;
  // the row's trace, 64 publishes at a time in LDS (loaded and waited for once per
  // chunk, for the reason above); the next publish in registers
  __shared__ int64_t s_ptk[kRowsPerWave * kTraceChunk];
  __shared__ int32_t s_prq[kRowsPerWave * kTraceChunk];
  int64_t* const ptk = s_ptk + (lane / kRowLanes) * kTraceChunk;
  int32_t* const prq = s_prq + (lane / kRowLanes) * kTraceChunk;
  auto stage_chunk = [&](int base) {  // publishes base .. base + 63 (row-uniform call)
    constexpr int kPer = kTraceChunk / kRowLanes;
    int64_t tk[kPer];
    int32_t rq[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {  // every load issued before any is used
      const int t = base + li + u * kRowLanes;
      const int tc = t < T ? t : T - 1;
      tk[u] = arrive[tc];
      rq[u] = reqs[tc];
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int q = li + u * kRowLanes;
      ptk[q] = base + q < T ? tk[u] : kNever;
      prq[q] = base + q < T ? rq[u] : 0;
    }
    // the row's lanes read each other's slots next: keep the compiler from
    // moving those LDS reads above these stores (valid in divergent code)
    __builtin_amdgcn_wave_barrier();
  };
  if (live && T > 0) stage_chunk(0);
  int64_t p_tick = (live && T > 0) ? ptk[0] : kNever;
  int32_t p_req = (live && T > 0) ? prq[0] : 0;
  // per-replication counts (32-bit: each is at most T, except events)
  uint32_t c_tasks = 0, c_local = 0, c_fwd = 0, c_acc = 0, c_rej = 0, c_drop = 0, c_nonodes = 0, c_relb = 0,
           c_infl = 0, c_reln = 0, c_relay = 0;
  uint64_t c_events = 0;
  uint32_t err = row_any<kRowLanes>(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;
  bool fin = !live || err != FOGNET_OK;  // row-uniform: this replication's loop has ended
  bad = false;
  int64_t end_tick = kNever;  // the last event dispatched (where an error ends the replication)
  uint32_t end_seq = ~0u;

  // (no `continue` inside: every path of a step falls through to its end, so the
  // loop-carried state needs no copies at extra loop exits)
#ifdef FOGNET_V2_PROF
  uint32_t pr_iter = 0u, pr_batch = 0u, pr_gen = 0u, pr_fire = 0u;  // profile build only
  uint64_t pr_t[4] = {0, 0, 0, 0}, pr_last = __builtin_amdgcn_s_memtime();
#define VTM(i)                                          \
  {                                                     \
    const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
    pr_t[i] += now_ - pr_last;                          \
    pr_last = now_;                                     \
  }
#else
#define VTM(i)
#endif
  while (ballot(!fin)) {
#ifdef FOGNET_V2_PROF
    ++pr_iter;
#endif
    if (!fin) {  // (finished rows wait for the others; their lanes stay off)
    // ---- a batch of simple timer firings (kBatchFirings): the earliest firings of the
    // row's nodes that come before every other pending event (H), before the first
    // firing that releases a reservation (K) and before the arrival of any advert a
    // firing of the batch queues (M), handled at once, each on its node's lane
    bool batched = false;
    if (kBatchFirings) {
      // H: the earliest event that draws sequence numbers or touches a node's state
      // (task arrivals, publishes) or the request list (the broker's RELEASERESOURCE)
      const int64_t ht = in_n ? in_hd.tick : kNever;
      const uint32_t hs = in_n ? in_hd.seq : ~0u;
      int64_t H_t = (int64_t)row_min_u64<kRowLanes>((uint64_t)ht);
      uint32_t H_s = row_min_u32<kRowLanes>(ht == H_t ? hs : ~0u);
      if (next < T && earlier32(p_tick, (uint32_t)N + (uint32_t)next, H_t, H_s)) {
        H_t = p_tick;
        H_s = (uint32_t)N + (uint32_t)next;
      }
      if (b_sched && earlier32(b_tick, b_seq, H_t, H_s)) {
        H_t = b_tick;
        H_s = b_seq;
      }
      VTM(0)
      const bool cand = t_sched && t_tick < stop && earlier32(t_tick, t_seq, H_t, H_s);
      // messages reaching the broker before H: adverts set the view, status-6 acks
      // relay and erase their request (BrokerBaseApp2.cc:128-154); they draw no
      // number and touch neither a node nor what a firing reads
      const bool arr = out_n && out_hd.tick < stop && earlier32(out_hd.tick, out_hd.seq, H_t, H_s);
      VTM(1)
      const uint32_t rowm = (uint32_t)((1ull << kRowLanes) - 1ull);
      const uint32_t rowb = (uint32_t)(ballot(cand) >> (lane & ~(kRowLanes - 1))) & rowm;
      const bool rowa = ((ballot(arr) >> (lane & ~(kRowLanes - 1))) & rowm) != 0ull;
      if (rowb && seq >= kSeqLimit) {
        err = FOGNET_ERR_CAPACITY;  // (32-bit insertion sequence)
        fin = true;
        batched = true;
      } else if (rowb || rowa) {
        batched = true;
        // Several periods per node (kBatchGens).  No task reaches a node before H, so
        // node j's firings in the batch are t_j + g P (g < G_j; every firing re-arms
        // 0.01 s later, ComputeBrokerApp2.cc:219), cut at H and, so that the batch is a
        // prefix of the FES order, at the row's first firing + kBatchGens periods.
        int64_t Hc_t = H_t;
        uint32_t Hc_s = H_s;
        if (rowb) {
          const int64_t cap =
              (int64_t)row_min_u64<kRowLanes>((uint64_t)(cand ? t_tick : kNever)) + kBatchGens * kAdvertPeriod;
          if (cap < Hc_t) {
            Hc_t = cap;
            Hc_s = 0u;  // (nothing at the cut's tick)
          }
        }
        // a later period's sequence number is drawn in the batch, after every pending
        // one, so at the cut's own tick only a first firing can precede it
        uint32_t G = 0u;
        if (cand) {
          int64_t tg = t_tick;
          while (G < (uint32_t)kBatchGens && tg < stop && (tg < Hc_t || (G == 0u && tg == Hc_t && t_seq < Hc_s))) {
            ++G;
            tg += kAdvertPeriod;
          }
        }
        // the periods that release a reservation (:222-226: the oldest, when its
        // deadline < now), peeked from the FIFO before any is popped
        uint32_t rmask = 0u;
        if (G && t_kind == kKindRelease && rs_n) {
          uint32_t k = 0u;
          V2Res h = rs_hd;
          for (uint32_t g = 0u; g < G && k < rs_n; ++g) {
            if (h.deadline < dbl(t_tick + (int64_t)g * kAdvertPeriod)) {
              rmask |= 1u << g;
              ++k;
              if (k < rs_n) {
                if (k == 1u) {
                  h = rs_nx;
                } else {
                  h = res[(rs_h + k) & qm];
                  sync_vm();
                }
              }
            }
          }
        }
        // The firings' order is (tick, period, first firing's sequence): at one tick a
        // first firing (pending sequence) precedes every later period (drawn in the
        // batch), and later periods of two nodes keep the order of their firings one
        // period before, down to the period where one of them is a first firing.  Each
        // firing draws two sequence numbers (its advert's, its next firing's), three
        // when it releases (its ack's first); off[g] counts those the firings before
        // period g of this node draw: node i's firings before it are its periods
        // g' < g + ceil((t_j - t_i) / P) (+1 for a same-tick one that precedes).
        uint32_t off[kBatchGens];
#pragma unroll
        for (int g = 0; g < kBatchGens; ++g) off[g] = 0u;
        uint32_t tot = 0u;
        const uint32_t grow = (uint32_t)(ballot(G != 0u) >> (lane & ~(kRowLanes - 1))) & rowm;
        const uint32_t gr = G | (rmask << 8);
        for (uint32_t m = grow; m; m &= m - 1u) {
          const int w = (int)__builtin_ctz(m);
          const uint32_t gw = row_bcast_u32<kRowLanes>(gr, w);
          const int64_t tw = (int64_t)row_bcast_u64<kRowLanes>((uint64_t)t_tick, w);
          const uint32_t sw = row_bcast_u32<kRowLanes>(t_seq, w);
          const int Gw = (int)(gw & 0xFFu);
          const uint32_t rw = gw >> 8;
          tot += 2u * (uint32_t)Gw + (uint32_t)__builtin_popcount(rw);
          if (G) {
            const int64_t d = t_tick - tw;  // |d| < kBatchGens P: exact in double
            int cd = (int)ceil((double)d / 1e10);
            if ((int64_t)cd * kAdvertPeriod == d && (cd < 0 || (cd == 0 && sw < t_seq))) ++cd;
#pragma unroll
            for (int g = 0; g < kBatchGens; ++g) {
              const int c = min(max(g + cd, 0), Gw);
              off[g] += 2u * (uint32_t)c + (uint32_t)__builtin_popcount(rw & ((1u << c) - 1u));
            }
          }
        }
        if ((uint64_t)seq + tot > (uint64_t)kSeqLimit) {
          err = FOGNET_ERR_CAPACITY;  // (32-bit insertion sequence)
          fin = true;
          G = 0u;
        }
        bool has_last = false;
        uint32_t n_rel = 0u;
#pragma unroll
        for (int g = 0; g < kBatchGens; ++g) {
          if ((uint32_t)g < G) {
            uint32_t sq = seq + off[g];
            const bool rl = (rmask >> g) & 1u;
            if (rl) {  // releaseResource: the oldest reservation, acked with status 6 (:225-235)
              const V2Res h = rs_hd;
              mips += h.req;  // :226
              ++rs_h;
              --rs_n;
              rs_hd = rs_nx;
              if (rs_n >= 2u) {
                rs_nx = res[(rs_h + 1u) & qm];
                sync_vm();
              }
              const V2MsgR m = {t_tick + ul, sq++, kMsgAck6, h.task, 0};
              if (out_n == Q) bad = true;
              else {
                if (out_n == 0u) out_hd = m;
                else if (out_n == 1u) out_nx = m;
                else outq[(out_h + out_n) & qm] = m;
                ++out_n;
              }
              O.done_tick[tbase + h.task] = t_tick;
              ++n_rel;
            }
            if (kPhantomAdverts && mips == last_sent && earlier32(ph_tick, ph_seq, t_tick, t_seq)) {
              // carries the value of the node's previous advert (kPhantomAdverts)
              ph_tick = t_tick + ul;
              ph_seq = sq;
              ph_cnt += ph_tick < stop ? 1u : 0u;
            } else {
              const V2MsgR m = {t_tick + ul, sq, kMsgAdvert, mips, 0};
              last_sent = mips;
              if (out_n == Q) bad = true;
              else {
                if (out_n == 0u) out_hd = m;
                else if (out_n == 1u) out_nx = m;
                else outq[(out_h + out_n) & qm] = m;
                ++out_n;
              }
            }
            if (off[g] + (rl ? 3u : 2u) == tot) {  // the batch's last firing (where an error would end the replication)
              has_last = true;
              end_tick = t_tick;
              end_seq = t_seq;
            }
            t_tick += kAdvertPeriod;
            t_seq = sq + 1u;
          }
        }
        const uint32_t nfire = (uint32_t)row_sum_i64<kRowLanes>((int64_t)G);
        if (nfire) {
          end_tick = (int64_t)row_min_u64<kRowLanes>((uint64_t)(has_last ? end_tick : kNever));
          end_seq = row_min_u32<kRowLanes>(has_last ? end_seq : ~0u);
        }
        // the messages (a queued advert of this batch's firings included: its arrival
        // commutes with them too)
        uint32_t n_arr = 0u, n_rl = 0u;
        while (!fin && out_n && out_hd.tick < stop && earlier32(out_hd.tick, out_hd.seq, H_t, H_s)) {
          if (out_hd.kind == kMsgAdvert) {
            view = out_hd.val;  // setMips (:132)
          } else if (list[out_hd.val] == kListForwarded) {  // ack 6: relay, erase if still listed (:145-153)
            list[out_hd.val] = kListNone;
            ++n_rl;
          }
          ++out_h;
          --out_n;
          out_hd = out_nx;
          if (out_n >= 2u) {
            out_nx = outq[(out_h + 1u) & qm];
            sync_vm();
          }
          ++n_arr;
        }
        const uint32_t na = (uint32_t)row_sum_i64<kRowLanes>((int64_t)n_arr);
        seq += tot;
        c_events += nfire + na;
        c_reln += (uint32_t)row_sum_i64<kRowLanes>((int64_t)n_rel);
        c_relay += (uint32_t)row_sum_i64<kRowLanes>((int64_t)n_rl);
#ifdef FOGNET_V2_PROF
        ++pr_batch;
        pr_fire += nfire;
#endif
        if (row_any<kRowLanes>(bad)) {
          err = FOGNET_ERR_CAPACITY;
          fin = true;
        }
      }
    }
    VTM(2)
    // then the earliest remaining event, in the same step (rows that batched take
    // their next event too: the union of the rows' paths is paid either way)
    (void)batched;
    {
#ifdef FOGNET_V2_PROF
    ++pr_gen;
#endif
    // ---- the earliest event: the lanes' own sources, then the broker's
    int64_t ct = kNever;
    uint32_t cs = ~0u;
    int src = 0;  // 1 self-message, 2 task arrival, 3 message at the broker
    if (t_sched) {
      ct = t_tick;
      cs = t_seq;
      src = 1;
    }
    if (in_n && earlier32(in_hd.tick, in_hd.seq, ct, cs)) {
      ct = in_hd.tick;
      cs = in_hd.seq;
      src = 2;
    }
    if (out_n && earlier32(out_hd.tick, out_hd.seq, ct, cs)) {
      ct = out_hd.tick;
      cs = out_hd.seq;
      src = 3;
    }
    const int64_t m_tick = (int64_t)row_min_u64<kRowLanes>((uint64_t)ct);
    const bool at = src != 0 && ct == m_tick;
    const uint32_t m_seq = row_min_u32<kRowLanes>(at ? cs : ~0u);  // same-tick events: insertion order decides
    const uint32_t wl = row_min_u32<kRowLanes>(at && cs == m_seq ? (uint32_t)li : 0xFFu);
    const int w = wl == 0xFFu ? 0 : (int)wl;
    int kind = wl == 0xFFu ? 0 : 1;  // 1 node-side event of lane w, 2 publish, 3 broker timer
    int64_t e_tick = kind ? m_tick : kNever;
    uint32_t e_seq = kind ? m_seq : ~0u;
    if (next < T) {
      if (earlier32(p_tick, (uint32_t)N + (uint32_t)next, e_tick, e_seq)) {
        e_tick = p_tick;
        e_seq = (uint32_t)N + (uint32_t)next;
        kind = 2;
      }
    }
    if (b_sched && earlier32(b_tick, b_seq, e_tick, e_seq)) {
      e_tick = b_tick;
      e_seq = b_seq;
      kind = 3;
    }
    if (kind == 0 || e_tick >= stop) fin = true;  // nothing left, or the sim-time-limit
    if (!fin && seq >= kSeqLimit) {
      err = FOGNET_ERR_CAPACITY;  // (32-bit insertion sequence)
      fin = true;
    }
    const int64_t now = e_tick;
    if (!fin) {
      ++c_events;
      end_tick = e_tick;
      end_seq = e_seq;
    }

    if (fin) {
    } else if (kind == 2 && (p_tick < prev_pub || p_tick > kMaxV2Tick)) {
      err = FOGNET_ERR_ARG;  // trace not sorted / out of range
      fin = true;
    } else if (kind == 2) {
      // ---- publish: BrokerBaseApp2.cc:176-195 + sendPubAck(:205-287)
      const int t = next++;
      prev_pub = p_tick;
      const int32_t req = p_req;
      if (next < T) {  // the following publish, in flight while this one is handled
        if ((next & (kTraceChunk - 1)) == 0) stage_chunk(next);
        p_tick = ptk[next & (kTraceChunk - 1)];
        p_req = prq[next & (kTraceChunk - 1)];
      }
      ++c_tasks;
      int32_t k = -1;
      uint32_t status;
      int64_t start = -1;
      uint8_t lmark = kListNone;
      if (req < pool) {  // :181 -> sendPubAck(true), :209-232
        pool -= req;
        lmark = kListLocal;
        status = FOGNET_V2_ST_LOCAL;
        start = now;
        ++c_local;
        b_sched = true;  // cancelEvent + scheduleAt(now + requiredTime) (:226-229)
        b_tick = now + rt_ticks;
        b_seq = seq++;
      } else if (N == 0) {  // :273-285: scheduleAt without cancelEvent
        status = FOGNET_V2_ST_NO_NODES;
        ++c_nonodes;
        if (b_sched) {
          err = FOGNET_ERR_STATE;  // "scheduleAt(): message already scheduled"
          fin = true;
        } else {
          b_sched = true;
          b_tick = now + rt_ticks;
          b_seq = seq++;
        }
      } else {
        // the LAST node whose advertised MIPS exceeds node 0's (:241-248), else node 0
        const int32_t v0 = (int32_t)row_bcast_u32<kRowLanes>((uint32_t)view, 0);
        k = (int32_t)((kRowLanes - 1u) - row_min_u32<kRowLanes>((kRowLanes - 1u) - ((own && li >= 1 && view > v0) ? (uint32_t)li : 0u)));
        const int32_t vk = (int32_t)row_bcast_u32<kRowLanes>((uint32_t)view, k);
        lmark = kListForwarded;  // :255-260, before the MIPS check
        if (req < vk) {          // :262-270: FognetMsgTask to node k
          status = FOGNET_V2_ST_FORWARDED;
          ++c_fwd;
          if (li == k) {
            const V2MsgR m = {now + dl, seq, req, t, 0};
            if (in_n == Q) {
              bad = true;
            } else {
              if (in_n == 0u) in_hd = m;
              else if (in_n == 1u) in_nx = m;
              else inq[(in_h + in_n) & qm] = m;
              ++in_n;
            }
          }
          ++seq;
          if (row_any<kRowLanes>(bad)) {
            err = FOGNET_ERR_CAPACITY;
            fin = true;
          }
        } else {
          status = FOGNET_V2_ST_DROPPED;
          ++c_drop;
        }
      }
      if (li == 0) {
        list[t] = lmark;
        O.node[tbase + t] = k;
        O.status[tbase + t] = (uint8_t)status;
        O.start_tick[tbase + t] = start;
        O.done_tick[tbase + t] = -1;
      }
    } else if (kind == 3) {
      // ---- broker RELEASERESOURCE: BrokerBaseApp2::releaseResource (:382-406), the
      // first request with deadline <= now (the oldest live one: deadlines follow
      // the list order), local or forwarded
      b_sched = false;
      int rel = -1;
      uint32_t mark = kListNone;
      if (li == 0) {
        while (list_h < next && list[list_h] == kListNone) ++list_h;
        if (list_h < next) {
          const double deadline = add_rn(dbl(arrive[list_h]), rt);
          if (deadline <= dbl(now)) {
            rel = list_h;
            mark = list[list_h];
            list[list_h] = kListNone;
            if (mark == kListLocal) O.done_tick[tbase + list_h] = now;
          }
        }
      }
      list_h = (int)row_bcast_u32<kRowLanes>((uint32_t)list_h, 0);
      rel = (int)row_bcast_u32<kRowLanes>((uint32_t)rel, 0);
      mark = row_bcast_u32<kRowLanes>(mark, 0);
      if (rel >= 0) {
        pool += reqs[rel];  // :386
        ++c_relb;
        if (mark == kListForwarded) ++c_infl;
      }
    } else {
      // ---- an event of node w
      const int wsrc = (int)row_bcast_u32<kRowLanes>((uint32_t)src, w);
      if (wsrc == 3) {
        // a node -> broker message reaches the broker (BrokerBaseApp2.cc:128-154)
        const int32_t mk = (int32_t)row_bcast_u32<kRowLanes>((uint32_t)out_hd.kind, w);
        const int32_t mv = (int32_t)row_bcast_u32<kRowLanes>((uint32_t)out_hd.val, w);
        if (li == w) {
          ++out_h;
          --out_n;
          out_hd = out_nx;
          if (out_n >= 2u) {
            out_nx = outq[(out_h + 1u) & qm];
            sync_vm();
          }
          if (mk == kMsgAdvert) view = mv;  // setMips (:132)
        }
        if (mk == kMsgAck6) {  // relay and erase the request if it is still listed (:145-153)
          bool relayed = false;
          if (li == 0 && list[mv] == kListForwarded) {
            list[mv] = kListNone;
            relayed = true;
          }
          if (row_any<kRowLanes>(relayed)) ++c_relay;
        }
      } else {
        // the node's own events: its self-message or a task arrival.  The owner
        // lane runs the handler; sequence numbers and per-task results are
        // broadcast afterwards (lane 0 of the row writes the outputs).
        int32_t o_task = -1;   // task whose result changed
        uint32_t o_what = 0u;  // 1 released, 2 accepted, 3 rejected
        uint32_t my_seq = seq;
        if (li == w) {
          if (wsrc == 1) {
            t_sched = false;
            if (t_kind == kKindRelease && rs_n) {
              // ComputeBrokerApp2::releaseResource (:222-245): the first reservation
              // with deadline < now (the oldest: deadlines follow arrival order)
              const V2Res h = rs_hd;
              if (h.deadline < dbl(now)) {
                mips += h.req;  // :226
                ++rs_h;
                --rs_n;
                rs_hd = rs_nx;
                if (rs_n >= 2u) {
                  rs_nx = res[(rs_h + 1u) & qm];
                  sync_vm();
                }
                o_task = h.task;
                o_what = 1u;
                const V2MsgR m = {now + ul, my_seq++, kMsgAck6, h.task, 0};  // puback 6 (:231-235)
                if (out_n == Q) bad = true;
                else {
                  if (out_n == 0u) out_hd = m;
                  else if (out_n == 1u) out_nx = m;
                  else outq[(out_h + out_n) & qm] = m;
                  ++out_n;
                }
              }
            }
            // advertiseMIPS (:202-220): advert, then the self-message again 0.01 s later
            if (kPhantomAdverts && mips == last_sent && earlier32(ph_tick, ph_seq, now, e_seq)) {
              // carries the value of the node's previous advert, which the broker already holds
              ph_tick = now + ul;
              ph_seq = my_seq++;
              ph_cnt += ph_tick < stop ? 1u : 0u;
            } else {
              const V2MsgR m = {now + ul, my_seq++, kMsgAdvert, mips, 0};
              last_sent = mips;
              if (out_n == Q) bad = true;
              else {
                if (out_n == 0u) out_hd = m;
                else if (out_n == 1u) out_nx = m;
                else outq[(out_h + out_n) & qm] = m;
                ++out_n;
              }
            }
            t_sched = true;
            t_tick = now + kAdvertPeriod;
            t_seq = my_seq++;
          } else {
            // ComputeBrokerApp2::processPacket, FognetMsgTask (:258-318)
            const int32_t t = in_hd.val;
            const int32_t req = in_hd.kind;
            ++in_h;
            --in_n;
            in_hd = in_nx;
            if (in_n >= 2u) {
              in_nx = inq[(in_h + 1u) & qm];
              sync_vm();
            }
            o_task = t;
            if (req < mips) {  // :269
              mips -= req;     // :272
              o_what = 2u;
              if (rs_n == Q) bad = true;
              else {
                const V2Res v = {t, req, add_rn(dbl(now), rt)};  // :274
                if (rs_n == 0u) rs_hd = v;
                else if (rs_n == 1u) rs_nx = v;
                else res[(rs_h + rs_n) & qm] = v;
                ++rs_n;
              }
              // cancelEvent + RELEASERESOURCE at now + requiredTime (:292-295)
              t_kind = kKindRelease;
              t_sched = true;
              t_tick = now + rt_ticks;
              t_seq = my_seq++;
            } else {
              o_what = 3u;  // TaskAck(false) (:299-306)
            }
          }
        }
        seq = row_bcast_u32<kRowLanes>(my_seq, w);
        o_task = (int32_t)row_bcast_u32<kRowLanes>((uint32_t)o_task, w);
        o_what = row_bcast_u32<kRowLanes>(o_what, w);
        if (row_any<kRowLanes>(bad)) {  // the replication ends here (nothing of this event is recorded)
          err = FOGNET_ERR_CAPACITY;
          fin = true;
          o_what = 0u;
        }
        if (o_what == 1u) {
          ++c_reln;
          if (li == 0) O.done_tick[tbase + o_task] = now;
        } else if (o_what == 2u) {
          ++c_acc;
          if (li == 0) {
            O.status[tbase + o_task] = FOGNET_V2_ST_ACCEPTED;
            O.start_tick[tbase + o_task] = now;
          }
        } else if (o_what == 3u) {
          ++c_rej;
          if (li == 0) O.status[tbase + o_task] = FOGNET_V2_ST_REJECTED;
        }
      }
    }
    }  // !batched
  }
  VTM(3)
  }

  // ---- tasks not published before the stop (or the error), and the record
  if (live) {
    for (int t = next + li; t < T; t += kRowLanes) {
      O.node[tbase + t] = -1;
      O.status[tbase + t] = 0;
      O.start_tick[tbase + t] = -1;
      O.done_tick[tbase + t] = -1;
    }
  }
  // unqueued adverts dispatched before the end (after an error: not the one still in flight)
  if (err != FOGNET_OK && ph_tick < stop && !earlier32(ph_tick, ph_seq, end_tick, end_seq)) ph_cnt -= 1u;
  c_events += (uint64_t)row_sum_i64<kRowLanes>(own ? (int64_t)ph_cnt : 0);
  const int64_t msum = row_sum_i64<kRowLanes>(own ? (int64_t)mips : 0);
  if (live && li == 0) {
    fognet_v2_stats st = {};
    st.n_tasks = c_tasks;
    st.n_local = c_local;
    st.n_forwarded = c_fwd;
    st.n_accepted = c_acc;
    st.n_rejected = c_rej;
    st.n_dropped = c_drop;
    st.n_no_nodes = c_nonodes;
    st.n_released_broker = c_relb;
    st.n_inflated = c_infl;
    st.n_released_node = c_reln;
    st.n_relayed = c_relay;
#ifdef FOGNET_V2_PROF
    st.n_no_nodes = pr_iter;
    st.n_dropped = pr_batch;
    st.n_inflated = pr_gen;
    st.n_rejected = pr_fire;
    st.n_local = pr_t[0];      // H (non-timer minimum)
    st.n_forwarded = pr_t[1];  // K, M
    st.n_accepted = pr_t[2];   // batch execution (rank, adverts)
    st.n_released_broker = pr_t[3];  // generic step
#endif
    st.events = (int64_t)c_events;
    st.node_mips_final_sum = msum;
    st.broker_mips_final = pool;
    st.status = (int32_t)err;
    O.stats[r] = st;
  }
}

}  // namespace

// queue rows per replication: 64 * the kernel's nodes per lane (the rows kernels use the first 64)
static size_t v2_rows(int32_t N) {
  const size_t npl = N <= kWave ? 1 : (size_t)1 << (32 - __builtin_clz((unsigned)((N + kWave - 1) / kWave - 1)));
  return npl * kWave;
}

size_t replay_v2_workspace_bytes(int32_t R, int32_t T, int32_t N, int32_t q_log2) {
  const size_t q = (size_t)R * v2_rows(N) << q_log2;
  return q * (2 * sizeof(V2Msg) + sizeof(V2Res)) + (size_t)R * (size_t)T;
}

hipError_t launch_replay_v2(const fognet_v2_in& in, const fognet_v2_out& out, void* ws, int32_t q_log2,
                            hipStream_t s) {
  if (in.R <= 0) return hipSuccess;
  V2Args a;
  a.in = in;
  a.out = out;
  a.q_log2 = q_log2;
  const size_t q = (size_t)in.R * v2_rows(in.N) << q_log2;
  a.inq = reinterpret_cast<V2Msg*>(ws);
  a.outq = a.inq + q;
  a.res = reinterpret_cast<V2Res*>(a.outq + q);
  a.list = reinterpret_cast<uint8_t*>(a.res + q);
  // rows of 16 lanes unless FOGNET_V2_ROW=32 (two replications per wavefront) or N > 16
  const char* rw = getenv("FOGNET_V2_ROW");
  const int row = (in.N > 16 || (rw && strcmp(rw, "32") == 0)) ? 32 : 16;
  // N <= 16: two replications per wavefront in rows 0-1 (rows 2-3 idle), i.e. two wavefronts
  // per SIMD at the C1 size: 375 -> 360 ms against all four rows of one wavefront busy
  // (FOGNET_V2_ACTIVE=4; one row per wavefront needs three generations of wavefronts at 164
  // VGPRs, 546 ms)
  const char* act = getenv("FOGNET_V2_ACTIVE");
  if (in.N <= 16 && row == 16 && act && strcmp(act, "4") == 0)
    hipLaunchKernelGGL(replay_v2_rows_kernel<16>, dim3((in.R + 3) / 4), dim3(kWave), 0, s, a);
  else if (in.N <= 16 && row == 16)
    hipLaunchKernelGGL((replay_v2_rows_kernel<16, 2>), dim3((in.R + 1) / 2), dim3(kWave), 0, s, a);
  else if (in.N <= 32)
    hipLaunchKernelGGL(replay_v2_rows_kernel<32>, dim3((in.R + 1) / 2), dim3(kWave), 0, s, a);
  else if (in.N <= 64)
    hipLaunchKernelGGL(replay_v2_kernel<1>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 128)
    hipLaunchKernelGGL(replay_v2_kernel<2>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 256)
    hipLaunchKernelGGL(replay_v2_kernel<4>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 512)
    hipLaunchKernelGGL(replay_v2_kernel<8>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 1024)
    hipLaunchKernelGGL(replay_v2_kernel<16>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 2048)
    hipLaunchKernelGGL(replay_v2_kernel<32>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 4096)
    hipLaunchKernelGGL(replay_v2_kernel<64>, dim3(in.R), dim3(kWave), 0, s, a);
  else if (in.N <= 8192)
    hipLaunchKernelGGL(replay_v2_kernel<128>, dim3(in.R), dim3(kWave), 0, s, a);
  else
    hipLaunchKernelGGL(replay_v2_kernel<256>, dim3(in.R), dim3(kWave), 0, s, a);
  return hipGetLastError();
}

}  // namespace fognet
