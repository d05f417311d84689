// replay_wide.hip — batched trace replay for large fog-node sets on gfx950
// (BASELINE.json configs[4], C5: 10,000 fog nodes; here N <= 65,536).  Same
// reference semantics and the same closed form as replay.hip,
// restated for node sets that do not fit in registers:
//   decision   BrokerBaseApp3::sendPubAck(status=false)   BrokerBaseApp3.cc:265-304
//   arrival    ComputeBrokerApp3::processPacket (task)     ComputeBrokerApp3.cc:269-320
//   completion ComputeBrokerApp3::releaseResource          ComputeBrokerApp3.cc:224-256
//   advert     advertiseMIPS + broker view update          ComputeBrokerApp3.cc:205-222,
//                                                          BrokerBaseApp3.cc:123-130
//
// One wavefront replays one replication.  Node j belongs to lane j % 64 (slot
// j / 64 of that lane) and only that lane reads or writes node j's state, so
// the loop needs no barriers:
//   HBM    view: per lane, its slots' next-advert tick (i64: the head
//          completion's advert reaches the broker; kNever: nothing pending)
//          and advertised busyTime (u32 seconds), slot-contiguous, so a group
//          of 16 slots is two cache lines of ticks and one of busy values;
//          WideEntry [R][T]: per task its arrival, completion, cumulative
//          service and the links of its node's pending chain;
//          WideNode [R][N]: chain ends + copies of head and tail fields (64 B).
//   LDS    per lane and group of 16 of its slots: earliest advert, its node,
//          smallest view key (busy << 32 | j); the lane's minima in VGPRs.
//          18 KiB at N = 10,000, so four replications share a CU (the loop is
//          latency-bound: every applied advert waits on HBM).
//   VGPRs  the record and parameters of the node the lane pushed to last
//          (the stale view keeps choosing it), written back when the lane
//          pushes to another node: a push issues no load.
// Publishes are decided one at a time in trace order: adverts that reached
// the broker strictly before the publish are applied first (lane-parallel:
// adverts of different nodes commute, those of one node come in completion
// order; an applied advert reloads its group's view with the node record and
// rescans it), the decision is a wave-wide u64 minimum of the lane minima (ties ->
// lowest index, the strict '<' of BrokerBaseApp3.cc:273), and the owner lane
// of the chosen node appends the task and accumulates its statistics (the
// same record replay.hip's fused epilogue writes).
//
// Node-down extension (A.down, fognet_hip.h; handleNodeCrash,
// ComputeBrokerApp3.cc:423-427): from its crash tick c on a node starts and
// completes nothing and drops arriving tasks (status 9).  A task's completion
// is kNever when it would start or finish at or after c, so its advert never
// becomes due and the broker keeps the node's last advert, as the reference
// does; lost tasks still join the node's chain so the pending count (and
// max_pending) follows the reference's `brokers` bookkeeping.
#include "replay_common.h"

namespace fognet {

namespace {

// Service seconds are any int / int (ComputeBrokerApp3.cc:276: up to 2^31 - 1).
// The tick arithmetic clamps them at kWideSCap: a task that is served with
// a service time (or a run prefix) of 2^22 s or more completes past kMaxTick
// (2^61 ticks = 26.7 days, 2^22 s = 48.5 days) and the replication is refused
// by the completion-tick check, so the clamp never changes a result; the
// cumulative service sums (advertised busy values) stay exact in 64 bits.
constexpr uint32_t kWideSCap = 1u << 22;
// Saturated advertised busy time in the 32-bit view (also the busy value of the
// view's slots past N, which never win: their index is larger).
constexpr uint32_t kBusySat = kViewBusySat;
// A start or completion tick at or past base + 2^22 s (beyond kMaxTick).
constexpr int64_t kPastRange = kMaxTick + 1;

// Per-lane minima are kept in two levels: for each group of kWideGroupSlots
// of the lane's slots the earliest pending advert, its node and the smallest
// view key live in LDS ([group][lane], conflict-free); the lane's overall
// minima in VGPRs.  An applied advert rescans one group and the group minima.
struct WideLds {
  int64_t* g_nxt;   // [G][64]
  int32_t* g_j;     // [G][64]
  uint64_t* g_key;  // [G][64]
  int64_t* g_w;     // [G][64] REF_V3 run horizon: smallest w (node_w) of the group
  uint32_t* hist;   // [FOGNET_HIST_METRICS][FOGNET_HIST_BINS]
  uint64_t* reg_key;  // [G] EXT_HIER: cached regional minimum key (valid per reg_valid)
  // EXT_HIER: escalated tasks decided but not yet pushed onto their node (slot per lane)
  int64_t* p_t;     // [64] publish tick
  int64_t* p_a;     // [64] arrival tick at the node
  int32_t* p_i;     // [64] task index (-1: free slot)
  int32_t* p_k;     // [64] node
  int32_t* p_r;     // [64] MIPSRequired
  // EXT_HIER: statistics inputs of pushed pending tasks, accumulated 64 at a time
  int64_t* q_t;     // [64] publish tick
  int64_t* q_a;     // [64] arrival tick
  int64_t* q_st;    // [64] start (kNever: never)
  int64_t* q_dn;    // [64] completion (kNever: never)
  int32_t* q_i;     // [64] task index
  uint32_t* q_sS;   // [64] service seconds << 3 | status (4, 5, 9 -> 4, 5, 1)
  // [G][64] per group of the lane: bit i (0-15) slot i has an advert pending (view tick
  // not kNever), bit 16 + i its advertised busy time is not 0 (past N: saturated).  An
  // advert rescans only the group's pending slots, and a key rescan of a group with a
  // zero-busy slot needs no view read (its smallest such slot holds the smallest key).
  uint32_t* g_msk;
  int G;
};

// EXT_HIER pending escalated tasks: one LDS slot per lane; past 64 in flight at
// once (decided within one hop latency of each other) they spill to an HBM
// overflow list (WideWs::ov_off, see flush_pending).
constexpr int kHierPending = kWave;

// Group minima in LDS up to 64 groups per lane (N <= 65,536, kWideMaxNodes); the flat
// policies above that (BIG) keep them in HBM, up to kWideBigMaxNodes (kGWords mask words).
constexpr int kWideLdsGroups = 64;
constexpr int kGWords = kWideBigMaxNodes / (kWave * kWideGroupSlots * 64);
static_assert(kGWords <= 32, "the summary of non-zero mask words is 32 bits");

// This lane's view in HBM: slot s (node s * 64 + lane) at [s].
struct WideView {
  int64_t* nxt;    // [G * kWideGroupSlots]
  uint32_t* busy;  // [G * kWideGroupSlots]
  int64_t* w;      // [G * kWideGroupSlots] REF_V3: node_w of the slot
};

// Node j lives in slot j >> 6 of lane (j + (j >> 10)) & 63: within each run of
// 1,024 nodes (one LDS group row, one EXT_HIER region) the lanes are rotated by
// the row index, so the rows' first nodes -- the smallest (busy, index) keys
// when the view is idle, i.e. the regional brokers' usual choices -- belong to
// different lanes, whose cached records then stay put (with lane j % 64 every
// region's first node was lane 0's: its one cached record thrashed).
// (FOGNET_POLICY_EXT_HIER only: the flat policies keep lane j % 64, measured 2 % faster there.)
template <bool R>
__host__ __device__ __forceinline__ int wlane(int j) { return R ? (j + (j >> 10)) & (kWave - 1) : j & (kWave - 1); }
template <bool R>
__host__ __device__ __forceinline__ int wnode(int s, int lane) {
  return R ? (s << 6) | ((lane - (s >> 4)) & (kWave - 1)) : (s << 6) | lane;
}
static_assert(kWave == 64 && kWideGroupSlots == 16, "wlane/wnode: 64 lanes, 16 slots (1,024 nodes) per group");

__host__ __device__ __forceinline__ int wide_groups(int N) {
  return ((N + kWave - 1) / kWave + kWideGroupSlots - 1) / kWideGroupSlots;
}

// Smallest view key (busy << 32 | node) of group g of this lane, from HBM
// (slot sl's busy just stored by this lane).  Slots past N hold busy
// 0xFFFFFFFF, above every admissible advertised busy time.
template <bool R>
__device__ __forceinline__ uint64_t group_key(const WideView& V, int lane, int g) {
  uint32_t b[kWideGroupSlots];
#pragma unroll
  for (int i = 0; i < kWideGroupSlots; ++i) b[i] = V.busy[g * kWideGroupSlots + i];
  uint64_t mk = ~0ull;
#pragma unroll
  for (int i = 0; i < kWideGroupSlots; ++i) {
    const uint64_t key = ((uint64_t)b[i] << 32) | (uint32_t)wnode<R>(g * kWideGroupSlots + i, lane);
    mk = key < mk ? key : mk;
  }
  return mk;
}

// group_key with the group's busy mask (WideLds::g_msk): a zero-busy slot holds
// the group's smallest key (nodes grow with the slot), else the full scan.
template <bool R>
__device__ __forceinline__ uint64_t group_key_m(const WideView& V, const WideLds& L, int lane, int g) {
  const uint32_t z = ~(L.g_msk[g * kWave + lane] >> 16) & 0xFFFFu;
  if (z) return (uint64_t)(uint32_t)wnode<R>(g * kWideGroupSlots + __builtin_ctz(z), lane);
  return group_key<R>(V, lane, g);
}

// The lane's earliest advert over its groups (first group on ties).
__device__ __forceinline__ void lane_min_nxt(const WideLds& L, int lane, int64_t& mn, int& mj) {
  mn = kNever;
  mj = lane;
#pragma unroll 4
  for (int g = 0; g < L.G; ++g) {
    const int64_t x = L.g_nxt[g * kWave + lane];
    const int jj = L.g_j[g * kWave + lane];
    if (x < mn) {
      mn = x;
      mj = jj;
    }
  }
}

// The lane's smallest view key over its groups.
__device__ __forceinline__ uint64_t lane_min_key(const WideLds& L, int lane) {
  uint64_t mk = ~0ull;
#pragma unroll 4
  for (int g = 0; g < L.G; ++g) {
    const uint64_t key = L.g_key[g * kWave + lane];
    mk = key < mk ? key : mk;
  }
  return mk;
}

// The lane's groups with a pending advert (the lane minima and the run horizon visit only
// these).  Up to 64 groups per lane (N <= 65,536): a bit mask in a register.  Above (BIG,
// the flat policies up to kWideBigMaxNodes, the group minima in HBM): kGWords mask words
// per lane in LDS ([word][lane]) and a register summary of the non-zero words.
template <bool BIG>
struct GroupSet {
  uint64_t m = 0ull;        // !BIG: bit g
  uint32_t sum = 0u;        // BIG: bit w: word w is not zero
  uint64_t* wl = nullptr;   // BIG: this lane's words, wl[w * kWave]
  __device__ __forceinline__ void set(int g, bool on) {
    if constexpr (!BIG) {
      m = on ? m | (1ull << g) : m & ~(1ull << g);
    } else {
      const int w = g >> 6;
      uint64_t x = wl[w * kWave];
      x = on ? x | (1ull << (g & 63)) : x & ~(1ull << (g & 63));
      wl[w * kWave] = x;
      sum = x ? sum | (1u << w) : sum & ~(1u << w);
    }
  }
  template <class F>
  __device__ __forceinline__ void each(F&& f) const {
    if constexpr (!BIG) {
      for (uint64_t x = m; x; x &= x - 1ull) f((int)__builtin_ctzll(x));
    } else {
      for (uint32_t s = sum; s; s &= s - 1u) {
        const int w = (int)__builtin_ctz(s);
        for (uint64_t x = wl[w * kWave]; x; x &= x - 1ull) f(w * 64 + (int)__builtin_ctzll(x));
      }
    }
  }
};

// The same over the groups with a pending advert only: the other groups hold kNever in
// both minima.
template <bool BIG>
__device__ __forceinline__ void lane_min_nxt_w_m(const WideLds& L, int lane, const GroupSet<BIG>& ga, int64_t& mn,
                                                 int& mj, int64_t& mw) {
  mn = kNever;
  mj = lane;
  mw = kNever;
  ga.each([&](int g) {
    const int64_t x = L.g_nxt[g * kWave + lane];
    const int jj = L.g_j[g * kWave + lane];
    const int64_t w = L.g_w[g * kWave + lane];
    if (x < mn) {
      mn = x;
      mj = jj;
    }
    mw = w < mw ? w : mw;
  });
}
template <bool BIG>
__device__ __forceinline__ void lane_min_nxt_m(const WideLds& L, int lane, const GroupSet<BIG>& ga, int64_t& mn,
                                               int& mj) {
  mn = kNever;
  mj = lane;
  ga.each([&](int g) {
    const int64_t x = L.g_nxt[g * kWave + lane];
    const int jj = L.g_j[g * kWave + lane];
    if (x < mn) {
      mn = x;
      mj = jj;
    }
  });
}

__device__ __forceinline__ void lane_min(const WideLds& L, int lane, int64_t& mn, int& mj, uint64_t& mk) {
  lane_min_nxt(L, lane, mn, mj);
  mk = lane_min_key(L, lane);
}

// ---- REF_V3 run horizon (the register kernel's horizon_all_in, restated per
// node so that it needs no knowledge of the current decision).
//
// Node j != k (k: the argmin, key best = busy_b << 32 | k) can change the
// decision only with an advert whose busy value v satisfies (v << 32 | j) <
// best, i.e. v <= busy_b.  While a run is pushed to k, j receives no task.
// If every pending task of j reached it before its head completes, its next
// advert (at nxt_j) carries v1 = tl_C - hd_C and each later one the service
// of the remaining tasks, so it drops by at most the seconds elapsed: an
// advert of j with v <= busy_b comes no earlier than nxt_j + (v1 - busy_b)
// seconds, and never earlier than nxt_j.  With
//   w_j = nxt_j + v1 s      (all arrived)      w_j = nxt_j  (tasks in flight)
// every such advert comes at or after max(nxt_j, w_j - busy_b s), so at or
// after max(min_j nxt_j, min_j w_j - busy_b s): the run may extend to that
// tick and to k's own next advert.  v1 is capped at 2^21 s (keeps the sum
// below 2^63); a cap, a stale (too small) group minimum or k's own entry only
// lower the bound, which shortens runs and never changes a decision.
__device__ __forceinline__ int64_t node_w(const WideNode& h, int64_t nxt, int64_t dl) {
  if (h.npend == 0 || nxt == kNever) return kNever;
  if (!arrives_before(h.tl_a, h.hd_done, dl, h.hd_S)) return nxt;
  const uint64_t v1 = h.tl_C - h.hd_C;
  return nxt + ticks_of((uint32_t)(v1 < ((uint64_t)1 << 21) ? v1 : ((uint64_t)1 << 21)));
}



// Workspace layout (launch_replay_wide, replay_wide_workspace_bytes).
struct WideWs {
  size_t e_off, nd_off, nxt_off, busy_off, w_off, dv_off, gm_off, gd_off, gu_off, ov_off, gx_off, bytes;
};

// BIG (group minima in HBM): per workspace slot [G][64] of g_nxt, g_key, g_w (8 B), g_j,
// g_msk (4 B): 2 KiB per group
constexpr size_t kGxGroupBytes = (size_t)kWave * (3 * sizeof(int64_t) + 2 * sizeof(int32_t));
__host__ __device__ __forceinline__ bool wide_big(int32_t N, bool force) {
  return force || wide_groups(N) > kWideLdsGroups;
}

__host__ __device__ __forceinline__ size_t align64(size_t x) { return (x + 63) & ~(size_t)63; }

// gen: + the generated node parameters (MIPS, dl, ul) of each slot
__host__ __device__ __forceinline__ WideWs wide_ws(int32_t R, int32_t T, int32_t N, bool gen, bool big) {
  const size_t SP = (size_t)wide_groups(N) * kWideGroupSlots;  // view slots per lane
  WideWs w;
  w.e_off = 0;
  w.nd_off = align64(w.e_off + (size_t)R * (size_t)T * sizeof(WideEntry));
  w.nxt_off = align64(w.nd_off + (size_t)R * (size_t)N * sizeof(WideNode));
  w.busy_off = align64(w.nxt_off + (size_t)R * kWave * SP * sizeof(int64_t));
  w.w_off = align64(w.busy_off + (size_t)R * kWave * SP * sizeof(uint32_t));
  w.dv_off = align64(w.w_off + (size_t)R * kWave * SP * sizeof(int64_t));
  w.gm_off = align64(w.dv_off + (size_t)R * (size_t)N * sizeof(uint64_t));
  const size_t RN = gen ? (size_t)R * (size_t)N : 0;
  w.gd_off = align64(w.gm_off + RN * sizeof(int32_t));
  w.gu_off = align64(w.gd_off + RN * sizeof(int64_t));
  // EXT_HIER: the pending-escalation overflow list, [R][T] task indices
  w.ov_off = align64(w.gu_off + RN * sizeof(int64_t));
  w.gx_off = align64(w.ov_off + (size_t)R * (size_t)T * sizeof(int32_t));
  w.bytes = align64(w.gx_off + (big ? (size_t)R * (size_t)wide_groups(N) * kGxGroupBytes : 0));
  return w;
}

// Generated mode's per-slot node parameters (workspace).
struct GenNodes {
  int32_t* m;
  int64_t* d;
  int64_t* u;
  uint64_t* dv;
};

template <int POL, bool BIG>
__device__ __forceinline__ void replay_wide_rep(const ReplayArgs& A, int r, int wr, WideEntry* E, WideNode* ND,
                                                int64_t* VN, uint32_t* VB, int64_t* VW, GenNodes GN, int32_t* OV,
                                                unsigned char* GX, const RegionWs& RW, unsigned char* w_lds);

// One replication per workgroup (r = blockIdx.x), or, with A.wide_list set,
// the replications the register kernel handed over, taken in turn by the
// workgroups (workspace slot = blockIdx.x); every workgroup leaves when the
// list (complete before this launch, stream order) is exhausted.
template <int POL, bool BIG>
__global__ __launch_bounds__(64) void replay_wide_kernel(ReplayArgs A, WideEntry* E, WideNode* ND, int64_t* VN,
                                                         uint32_t* VB, int64_t* VW, GenNodes GN, int32_t* OV,
                                                         unsigned char* GX, RegionWs RW) {
  extern __shared__ __align__(16) unsigned char w_lds[];
  if (A.wide_list == nullptr) {
    replay_wide_rep<POL, BIG>(A, blockIdx.x, blockIdx.x, E, ND, VN, VB, VW, GN, OV, GX, RW, w_lds);
    return;
  }
  const int n = *A.wide_count;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    replay_wide_rep<POL, BIG>(A, A.wide_list[i], blockIdx.x, E, ND, VN, VB, VW, GN, OV, GX, RW, w_lds);
    __syncthreads();  // LDS reuse by the next replication
  }
}

// Replication r with workspace slot wr.
template <int POL, bool BIG>
__device__ __forceinline__ void replay_wide_rep(const ReplayArgs& A, int r, int wr, WideEntry* E, WideNode* ND,
                                                int64_t* VN, uint32_t* VB, int64_t* VW, GenNodes GN, int32_t* OV,
                                                unsigned char* GX, const RegionWs& RW, unsigned char* w_lds) {
  constexpr bool kExt = POL == FOGNET_POLICY_EXT_LAT;
  constexpr bool kHier = POL == FOGNET_POLICY_EXT_HIER;
  static_assert(!(BIG && kHier), "EXT_HIER keeps its regions (groups) in LDS");
  constexpr bool kPerPublish = kExt || kHier;  // the decision depends on the publish itself
  const int lane = threadIdx.x;
  const int T = A.T, N = A.N;
  WideLds L;
  L.G = wide_groups(N);
  // group minima: LDS, or (BIG) this workspace slot's [G][64] arrays in HBM
  unsigned char* const gbase = BIG ? GX + (size_t)wr * (size_t)L.G * kGxGroupBytes : w_lds;
  L.g_nxt = reinterpret_cast<int64_t*>(gbase);
  L.g_key = reinterpret_cast<uint64_t*>(L.g_nxt + L.G * kWave);
  L.g_w = reinterpret_cast<int64_t*>(L.g_key + L.G * kWave);
  L.g_j = reinterpret_cast<int32_t*>(L.g_w + L.G * kWave);
  L.hist = BIG ? reinterpret_cast<uint32_t*>(w_lds) : reinterpret_cast<uint32_t*>(L.g_j + L.G * kWave);
  L.reg_key = reinterpret_cast<uint64_t*>(L.hist + FOGNET_HIST_METRICS * FOGNET_HIST_BINS);
  L.p_t = reinterpret_cast<int64_t*>(L.reg_key + (BIG ? 0 : L.G));
  L.p_a = L.p_t + kHierPending;
  L.p_i = reinterpret_cast<int32_t*>(L.p_a + kHierPending);
  L.p_k = L.p_i + kHierPending;
  L.p_r = L.p_k + kHierPending;
  L.q_t = reinterpret_cast<int64_t*>(L.p_r + kHierPending);
  L.q_a = L.q_t + kWave;
  L.q_st = L.q_a + kWave;
  L.q_dn = L.q_st + kWave;
  L.q_i = reinterpret_cast<int32_t*>(L.q_dn + kWave);
  L.q_sS = reinterpret_cast<uint32_t*>(L.q_i + kWave);
  L.g_msk = BIG ? reinterpret_cast<uint32_t*>(L.g_j + L.G * kWave) : L.q_sS + kWave;
  // BIG: the active-group mask words after the other LDS arrays ([kGWords][64])
  uint64_t* const gw_lds = reinterpret_cast<uint64_t*>(BIG ? reinterpret_cast<unsigned char*>(L.q_sS + kWave) : w_lds);
  const int SP = L.G * kWideGroupSlots;
  const WideView V{VN + ((size_t)wr * kWave + lane) * SP, VB + ((size_t)wr * kWave + lane) * SP,
                   VW + ((size_t)wr * kWave + lane) * SP};
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  WideEntry* const e = E + (size_t)wr * (size_t)T;
  int32_t* const ov = OV + (size_t)wr * (size_t)T;  // EXT_HIER pending-escalation overflow list
  WideNode* const nd = ND + (size_t)wr * (size_t)N;
  const bool hist = A.hist != nullptr;
  // generated mode (ReplayArgs::gen_on): the node parameters are computed
  // into this slot's workspace, the trace 64 publishes at a time
  const bool gen = A.gen_on != 0;
  GenRep g{};
  if (gen) g = gen_rep(A.gen, A.gen_r0 + r, r);
  const size_t sbase = (size_t)wr * (size_t)N;
  const int32_t* const P_mips = gen ? GN.m + sbase : A.mips + nbase;
  const int64_t* const P_dl = gen ? GN.d + sbase : A.dl + nbase;
  const int64_t* const P_ul = gen ? GN.u + sbase : A.ul + nbase;
  const int64_t arrive0 = gen ? kNever : (T > 0 ? A.arrive[tbase] : kNever);
  uint64_t ul_max = 0u;

  // ---- node parameters + preconditions (fognet_hip.h, fognet_batch_in);
  // every node's first advert {MIPS, busyTime = 0.0} has reached the broker
  bool bad = false;
  for (int sj = 0; sj < SP; ++sj) {  // this lane's nodes
    const int j = wnode<kHier>(sj, lane);
    if (j >= N) continue;
    int32_t m;
    int64_t d, u, ia;
    if (gen) {
      gen_node(g, j, m, d, u);
      ia = u;
      GN.m[sbase + j] = m;  // read back by this lane only (node j's owner)
      GN.d[sbase + j] = d;
      GN.u[sbase + j] = u;
      ul_max = (uint64_t)u > ul_max ? (uint64_t)u : ul_max;
    } else {
      m = A.mips[nbase + j];
      d = A.dl[nbase + j];
      u = A.ul[nbase + j];
      ia = A.init[nbase + j];
    }
    const int64_t dn = A.down ? A.down[nbase + j] : kNever;
    bad |= (m <= 0) | (d < 0) | (u < 0) | (d > kMaxTick) | (u > kMaxTick) | (ia < u) | (ia >= arrive0);
    bad |= dn != kNever && (dn < ia || dn > kMaxTick);
    if constexpr (kExt) bad |= d >= kExtMaxDl;
    nd[j] = WideNode{-1, -1, 0, -1, 0, 0u, 0, 0, 0u, 0u, 0u};
    const UDiv dv = udiv_magic((uint32_t)(m > 0 ? m : 1));
    GN.dv[sbase + j] = (uint64_t)dv.m | ((uint64_t)dv.sh << 32);
  }
  for (int s = 0; s < SP; ++s) {  // slots past N too (group rescans read them): never due, never chosen
    V.nxt[s] = kNever;
    V.busy[s] = wnode<kHier>(s, lane) < N ? 0u : 0xFFFFFFFFu;
    if constexpr (!kPerPublish) V.w[s] = kNever;
  }
  for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave) L.hist[h] = 0u;
  L.p_i[lane] = -1;  // EXT_HIER pending slots: free
  for (int g = 0; g < L.G; ++g) {  // the initial view: nothing pending, every busy 0
    const int j0 = wnode<kHier>(g * kWideGroupSlots, lane);  // the lane's smallest node of the group
    L.g_nxt[g * kWave + lane] = kNever;
    L.g_w[g * kWave + lane] = kNever;
    L.g_j[g * kWave + lane] = j0;
    L.g_key[g * kWave + lane] = j0 < N ? (uint64_t)(uint32_t)j0 : ~0ull;
    uint32_t nz = 0u;  // slots past N: busy saturated
    for (int i = 0; i < kWideGroupSlots; ++i) nz |= wnode<kHier>(g * kWideGroupSlots + i, lane) < N ? 0u : 1u << i;
    L.g_msk[g * kWave + lane] = nz << 16;
  }
  __syncthreads();
  uint32_t err = ballot(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;
  int64_t gen_carry = gen ? (int64_t)~wave_min_u64(~ul_max) + 1 : 0;

  int64_t mn;
  int mj;
  uint64_t mk;
  lane_min(L, lane, mn, mj, mk);
  GroupSet<BIG> gact;  // the lane's groups with a pending advert (lane minima visit only these)
  if constexpr (BIG) {
    gact.wl = gw_lds + lane;
    for (int w = 0; w < kGWords; ++w) gact.wl[w * kWave] = 0ull;
  }
  int64_t mw = kNever;  // REF_V3 run horizon: this lane's smallest node_w
  Acc acc = acc_identity();
  AbortPt ab = abort_none();  // the reference's abort point (replay_common.h)
  uint32_t max_pend = 0u;  // over this lane's nodes
  int n_short = 0;         // tasks of this lane's nodes that never complete (node-down)
  int64_t prev_t = INT64_MIN;
  int n_done = 0;
  // ---- EXT_HIER resume (replay_region.hip): a replication whose first escalated publish esc the
  // region passes found continues from the second pass's state there -- node records and
  // chains (sorted positions renamed to trace indices), advertised busy views, the finish
  // kernel's statistics record of the publishes before esc -- at publish esc, as if this kernel
  // had replayed them (until esc every decision is its region's, made from its region's view)
  int c_first = 0;
  if constexpr (kHier) {
    const int32_t esc = RW.esc != nullptr && !gen ? RW.esc[r] : 0;
    if (esc > 0 && esc < T && err == FOGNET_OK) {
      c_first = esc;
      const int32_t* const sidx = RW.s_idx + tbase;
      auto ren = [&](int32_t x) -> int32_t { return x < 0 || x >= T ? x : sidx[x]; };
      const WideEntry* const re = RW.e + tbase;
      for (int p = lane; p < T; p += kWave) {  // the entries of the publishes before esc
        const int32_t i = sidx[p];
        if (i < esc) {
          WideEntry x = re[p];
          x.prev = ren(x.prev);
          x.next = ren(x.next);
          e[i] = x;
        }
      }
      const WideNode* const rn = RW.nd + (size_t)r * (size_t)N;
      const uint32_t* const rvb = RW.vb + (size_t)r * (size_t)RW.B * FOGNET_HIER_REGION_NODES;
      for (int sj = 0; sj < SP; ++sj) {  // this lane's nodes: records and views
        const int j = wnode<kHier>(sj, lane);
        if (j >= N) continue;
        WideNode h = rn[j];
        h.hd = ren(h.hd);
        h.tl = ren(h.tl);
        h.hd_next = ren(h.hd_next);
        nd[j] = h;
        V.nxt[sj] = h.npend > 0 && h.hd_done != kNever ? h.hd_done + P_ul[j] : kNever;
        V.busy[sj] = rvb[j];  // (region j / 1024, its node j % 1024 at [slot][lane] = j % 1024)
      }
      for (int g = 0; g < L.G; ++g) {  // the group minima (regions) from the lane's views
        int64_t gmn = kNever;
        int gsi = 0;
        uint32_t gm = 0u;
        for (int i = 0; i < kWideGroupSlots; ++i) {
          const int64_t x = V.nxt[g * kWideGroupSlots + i];
          gm |= (x != kNever ? 1u : 0u) << i;
          gm |= (V.busy[g * kWideGroupSlots + i] != 0u ? 1u : 0u) << (16 + i);
          if (x < gmn) {
            gmn = x;
            gsi = i;
          }
        }
        L.g_nxt[g * kWave + lane] = gmn;
        L.g_j[g * kWave + lane] = wnode<kHier>(g * kWideGroupSlots + (gmn == kNever ? 0 : gsi), lane);
        L.g_msk[g * kWave + lane] = gm;
        L.g_key[g * kWave + lane] = group_key<kHier>(V, lane, g);
        gact.set(g, (gm & 0xFFFFu) != 0u);
      }
      if (lane == 0) {
        const unsigned char* const pr = RW.pacc + (size_t)r * kRegionResumeBytes;
        acc = *reinterpret_cast<const Acc*>(pr);
        ab = *reinterpret_cast<const AbortPt*>(pr + sizeof(Acc));
      }
      const uint32_t mp_b = lane < RW.B ? (uint32_t)RW.rec[(size_t)r * RW.B + lane].max_pend : 0u;
      const uint32_t mp_r = ~wave_min_u32(~mp_b);  // (all lanes: a cross-lane reduction)
      max_pend = lane == 0 ? mp_r : 0u;
      n_done = esc;
      prev_t = A.arrive[tbase + esc - 1];
      __threadfence_block();
      __syncthreads();  // (the entries and records written above are read by their nodes' lanes)
      lane_min(L, lane, mn, mj, mk);
    }
  }
  // the node this lane pushed to last: under the stale view the broker keeps
  // choosing it, so its record and parameters stay in registers between
  // pushes; nd[cj] in HBM is stale until the record is written back (when
  // the lane pushes to another node, and after the loop)
  int cj = -1;
  WideNode ch{};
  int32_t c_mips = 1;
  uint64_t c_dv = 1ull;
  int64_t c_dl = 0, c_ul = 0, c_down = kNever;

  // record and parameters of node kk into its owner lane's cache
  auto cache_node = [&](uint32_t kk) {
    if (lane == wlane<kHier>((int)kk) && (int)kk != cj) {
      if (cj >= 0) nd[cj] = ch;  // write back the previous node's record
      cj = (int)kk;
      ch = nd[kk];
      c_mips = P_mips[kk];
      c_dv = GN.dv[sbase + kk];
      c_dl = P_dl[kk];
      c_ul = P_ul[kk];
      c_down = A.down ? A.down[nbase + kk] : kNever;
    }
  };

  // ---- FOGNET_POLICY_EXT_HIER: an escalated task takes the extra hop, so a
  // direct task decided after it can reach the same node first; the node serves
  // in arrival order.  Escalated tasks therefore wait in the pending slots
  // (LDS, one per lane) and are pushed onto their node's chain only once every
  // task that reaches the node no later than them has been pushed: before a
  // direct task to the node with a later (or the same) arrival, before the
  // adverts of a publish tick past their arrival (whose completions they may
  // precede), and at the end.  Each chain stays in arrival order, so the FIFO
  // recurrence and the advert scans hold as for direct tasks.  A pushed pending
  // task's statistics and outputs are recorded at once (uniform code).
  // Overflow (ComputeBrokerApp3.cc:305-309: a node's FIFO takes any number of
  // tasks, so any number may be in flight): while all 64 slots are taken, or
  // the overflow list is not empty, an escalated task i goes to the HBM list
  // ov[ov_head .. ov_tail) (decision order, -1: pushed already) with its
  // pending fields in its own entry e[i] (written for real when it is pushed:
  // {a, done := publish tick, S := MIPSRequired, prev := node, pad = 2}).
  // Every slot's task was decided before every listed one, so pushing the
  // slots' selected tasks first and then the list's in list order keeps each
  // node's arrival order (per node decision order: the same dl and hop).
  int n_pend = 0;  // pending escalated tasks, slots and overflow list (wave-uniform)
  int n_ovf = 0;   // of which in the overflow list (wave-uniform)
  int ov_head = 0, ov_tail = 0;
  int n_sq = 0;    // staged statistics of pushed pending tasks (wave-uniform)
  // accumulate the staged statistics, one task per lane (the chunk end's code)
  auto drain_stats = [&]() {
    if (lane < n_sq) {
      const int64_t t_q = L.q_t[lane], a_q = L.q_a[lane], st_q = L.q_st[lane], dn_q = L.q_dn[lane];
      const int32_t i_q = L.q_i[lane];
      const uint32_t sS = L.q_sS[lane];
      const uint32_t status_q = sS & 7u, S_q = sS >> 3;  // (S only feeds busy_s: < 2^29 here, see push_one)
      if (dn_q != kNever) {
        acc_task(acc, ab, t_q, a_q, st_q, dn_q, S_q, status_q, i_q, hist ? L.hist : nullptr);
        if (hist) atomicAdd(&L.hist[FOGNET_HIST_BINS + hist_bin(dn_q - t_q)], 1u);
      } else {  // node-down
        n_short += 1;
        if (status_q == 5u) acc.n5 += 1u;
        if (status_q == 4u) {
          acc.n4 += 1u;
          if (st_q != kNever) acc_qtime(acc, ab, st_q, a_q, i_q, hist ? L.hist : nullptr);
        }
      }
    }
    n_sq = 0;
  };
  auto pend_count = [&](uint32_t kk) -> uint32_t {
    if (!n_pend) return 0u;
    uint32_t c = (uint32_t)__popcll(ballot(L.p_i[lane] >= 0 && (uint32_t)L.p_k[lane] == kk));
    for (int w0 = n_ovf ? ov_head : ov_tail; w0 < ov_tail; w0 += kWave) {
      const int pos = w0 + lane;
      const int32_t oi = pos < ov_tail ? ov[pos] : -1;
      c += (uint32_t)__popcll(ballot(oi >= 0 && (uint32_t)e[oi].prev == kk));
    }
    return c;
  };
  // push escalated task i (publish tick t_i, MIPSRequired req_i) onto node kk; false: past kMaxTick
  auto push_one = [&](int i, int64_t t_i, uint32_t req_i, uint32_t kk) -> bool {
    cache_node(kk);
    const int kl = wlane<kHier>((int)kk);
    const UDiv div_k{readlane_u32((uint32_t)c_dv, kl), readlane_u32((uint32_t)(c_dv >> 32), kl)};
    const int64_t dl_k = readlane_i64(c_dl, kl) + A.hier_up;  // (the hop, then the downlink)
    const int64_t ul_k = readlane_i64(c_ul, kl), down_k = readlane_i64(c_down, kl);
    const int32_t tl = (int32_t)readlane_u32((uint32_t)ch.tl, kl);
    const int64_t tl_done = readlane_i64(ch.tl_done, kl);
    const uint64_t tl_C = (uint64_t)readlane_i64((int64_t)ch.tl_C, kl);
    const uint32_t tl_S = readlane_u32(ch.tl_S, kl) & 0x7FFFFFFFu;
    const int64_t base_done = tl >= 0 ? tl_done : INT64_MIN;
    const uint32_t S = udiv(req_i, div_k);  // double tskTime = requiredMIPS / MIPS (ComputeBrokerApp3.cc:276)
    const int64_t a = t_i + dl_k;
    const uint64_t C = tl_C + S;
    int64_t start = kNever, done = kNever;
    uint32_t status = FOGNET_TASK_LOST;
    if (base_done != kNever) {  // FIFO: start = max(arrival, previous completion)
      const int64_t st = a > base_done ? a : base_done;
      const int64_t dn = S < kWideSCap ? st + ticks_of(S) : kPastRange;
      if (a < down_k) {
        if (base_done < a) status = 5u;
        else if (base_done > a) status = 4u;
        else status = dl_k < (int64_t)min(tl_S, kWideSCap) * kTicksPerSecond ? 5u : 4u;
        start = st < down_k ? st : kNever;
        done = dn < down_k ? dn : kNever;
      }
    } else if (a < down_k) {
      status = 4u;
    }
    if (a > kMaxTick || (done != kNever && done > kMaxTick)) return false;
    if (lane == 0) e[i] = WideEntry{a, done, C, S, tl, -1, 1};
    if (lane == kl) {
      WideNode h = ch;
      if (h.npend == 0) {  // the node's head: its advert is the node's next one
        h.hd = i;
        h.hd_done = done;
        h.hd_C = C;
        h.hd_S = S;
        const int64_t x = done == kNever ? kNever : done + ul_k;
        const int g = ((int)kk / kWave) / kWideGroupSlots;
        V.nxt[kk / kWave] = x;
        if (x != kNever) {
          L.g_msk[g * kWave + lane] |= 1u << ((kk / kWave) % kWideGroupSlots);
          gact.set(g, true);
        }
        if (x < L.g_nxt[g * kWave + lane]) {
          L.g_nxt[g * kWave + lane] = x;
          L.g_j[g * kWave + lane] = (int)kk;
        }
        if (x < mn) {
          mn = x;
          mj = (int)kk;
        }
      } else if (h.npend >= 2) {
        e[h.tl].next = i;
      }
      if (h.npend == 1) h.hd_next = i;  // the tail is the head (hoisted: DESIGN.md §3.6 "The hd_next miscompile")
      h.tl = i;
      h.tl_a = a;
      h.tl_done = done;
      h.tl_C = C;
      h.tl_S = S | 0x80000000u;  // escalated
      h.npend += 1;
      ch = h;
    }
    if (lane == 0 && !A.no_task_out) {
      const size_t o = tbase + (size_t)i;
      A.out_node[o] = (int32_t)kk;
      A.out_status[o] = (uint8_t)status;
      A.out_start[o] = start == kNever ? -1 : start;
      A.out_done[o] = done == kNever ? -1 : done;
    }
    // its statistics: staged, accumulated 64 tasks at a time (drain_stats), like the chunk's
    if (n_sq == kWave) drain_stats();
    if (lane == n_sq) {
      L.q_t[lane] = t_i;
      L.q_a[lane] = a;
      L.q_st[lane] = start;
      L.q_dn[lane] = done;
      L.q_i[lane] = i;
      L.q_sS[lane] = (min(S, 0x1FFFFFFFu) << 3) | (status & 7u);
    }
    ++n_sq;
    return true;
  };
  // push the pending tasks of node kk arriving at or before lim (by_node), or of any
  // node arriving before lim, in decision order (per node also arrival order)
  auto flush_pending = [&](bool by_node, uint32_t kk, int64_t lim) -> bool {
    while (n_pend - n_ovf > 0) {  // the slots
      const int32_t pi = L.p_i[lane];
      const int64_t pa = L.p_a[lane];
      const bool sel = pi >= 0 && (by_node ? ((uint32_t)L.p_k[lane] == kk && pa <= lim) : pa < lim);
      const uint32_t mi = wave_min_u32(sel ? (uint32_t)pi : ~0u);
      if (mi == ~0u) break;
      const int sl = (int)__builtin_ctzll(ballot(sel && (uint32_t)pi == mi));
      const int64_t t_i = readlane_i64(L.p_t[lane], sl);
      const uint32_t k_i = readlane_u32((uint32_t)L.p_k[lane], sl);
      const uint32_t r_i = readlane_u32((uint32_t)L.p_r[lane], sl);
      if (lane == sl) L.p_i[lane] = -1;
      --n_pend;
      if (!push_one((int)mi, t_i, r_i, k_i)) return false;
    }
    if (!n_ovf) return true;
    // the overflow list, 64 entries at a time, in list (= decision) order
    for (int w0 = ov_head; w0 < ov_tail && n_ovf; w0 += kWave) {
      const int pos = w0 + lane;
      const int32_t oi = pos < ov_tail ? ov[pos] : -1;
      WideEntry x{};
      if (oi >= 0) x = e[oi];
      uint64_t sm = ballot(oi >= 0 && (by_node ? ((uint32_t)x.prev == kk && x.a <= lim) : x.a < lim));
      while (sm) {
        const int sl = (int)__builtin_ctzll(sm);
        sm &= sm - 1ull;
        const int32_t i = (int32_t)readlane_u32((uint32_t)oi, sl);
        const int64_t t_i = readlane_i64(x.done, sl);
        const uint32_t k_i = readlane_u32((uint32_t)x.prev, sl);
        const uint32_t r_i = readlane_u32(x.S, sl);
        if (lane == sl) ov[pos] = -1;
        --n_ovf;
        --n_pend;
        if (!push_one((int)i, t_i, r_i, k_i)) return false;
      }
    }
    if (!n_ovf) {
      ov_head = ov_tail = 0;
    } else {  // drop the pushed entries at the head
      for (;;) {
        const int pos = ov_head + lane;
        const uint64_t live = ballot(pos < ov_tail && ov[pos] >= 0);
        if (live) {
          ov_head += (int)__builtin_ctzll(live);
          break;
        }
        ov_head += kWave;
      }
    }
    return true;
  };

#ifdef FOGNET_WIDE_PROF
  // profile build only (tools/wide_prof.py): loop counters, written over the statistics
  uint64_t pf_iter = 0, pf_advit = 0, pf_adv = 0, pf_same = 0, pf_hit = 0, pf_gkey = 0, pf_scan = 0, pf_runs = 0;
  uint64_t pf_t[7] = {0, 0, 0, 0, 0, 0, 0};  // s_memtime ticks per segment (WTM)
  uint32_t pf_walk = 0u;                      // backward walks of the adverts (+ steps << 16)
#define PF_WALK (&pf_walk)
  uint64_t pf_last = __builtin_amdgcn_s_memtime();
#define WTM(i)                                          \
  {                                                     \
    const uint64_t now_ = __builtin_amdgcn_s_memtime(); \
    pf_t[i] += now_ - pf_last;                          \
    pf_last = now_;                                     \
  }
#else
#define WTM(i)
#define PF_WALK nullptr
#endif
  // the decision is recomputed only after an advert changed the view
  // (adverts are the only view updates, BrokerBaseApp3.cc:123-130)
  bool view_changed = true;
  uint32_t k = 0u;
  uint64_t k_key = 0ull;  // REF_V3: the decision's view key (busy << 32 | k)
  uint64_t reg_valid = 0ull, glob_key = 0ull;  // EXT_HIER decision cache (regions < 64)
  uint64_t reg_dirty = 0ull;                   // regions with an advert applied since the last decision
  bool glob_valid = false;

  int64_t gen_t0 = 0;  // generated EXT_HIER: the first publish's tick (the mobility model's origin)
  for (int c0 = c_first; c0 < T && err == FOGNET_OK; c0 += kWave) {
    const int cnt = min(kWave, T - c0);
    const bool live = lane < cnt;
    // this chunk's pushed tasks, one per lane (publish c0 + lane): their
    // statistics are accumulated once per chunk with every pushed lane at once,
    // not run by run (a per-publish policy pushes one lane per iteration)
    // (and their per-task outputs are stored then, coalesced)
    bool q_on = false;
    int64_t q_a = 0, q_start = 0, q_done = 0;
    uint32_t q_S = 0u, q_status = 0u, q_k = 0u;
    int64_t ca;
    int32_t cr;
    if (gen) {
      gen_chunk(g, c0, T, lane, gen_carry, ca, cr);
    } else {
      ca = live ? A.arrive[tbase + c0 + lane] : kNever;
      cr = live ? A.req[tbase + c0 + lane] : 0;
    }
    int32_t cg = 0;  // EXT_HIER: the publish's regional broker (region = group of the LDS minima)
    if constexpr (kHier) {
      if (gen) {  // generated: the mobility model (replay_common.h gen_region) from the first publish's tick
        if (c0 == 0) gen_t0 = readlane_i64(ca, 0);
        cg = live ? gen_region(c0 + lane, ca, gen_t0, L.G) : 0;
      } else {
        cg = live ? A.region[tbase + c0 + lane] : 0;
      }
    }
    // trace preconditions: nondecreasing ticks, requirement >= 0, ticks < 2^61
    const int64_t prv = dpp_or_i64<kDppWaveShr1>(prev_t, ca);  // lane 0 gets prev_t
    if (ballot(live && (ca < prv || cr < 0 || ca > kMaxTick || (kHier && (cg < 0 || cg >= L.G))))) {
      err = FOGNET_ERR_ARG;
      break;
    }
    prev_t = readlane_i64(ca, cnt - 1);

    int jp = 0;
    WTM(6)
    while (jp < cnt) {
      const int64_t t = readlane_i64(ca, jp);
      if constexpr (kHier) {  // escalated tasks that reached their node before t (before any advert of t)
        if (n_pend && !flush_pending(false, 0u, t)) {
          err = FOGNET_ERR_ARG;
          break;
        }
      }

      // 1) completion adverts that reached the broker strictly before t
      bool lerr = false, lbroken = false;
      if (ballot(mn < t)) view_changed = true;
#ifdef FOGNET_WIDE_PROF
      ++pf_iter;
#endif
      while (ballot(mn < t)) {
#ifdef FOGNET_WIDE_PROF
        ++pf_advit;
        pf_adv += (uint64_t)__popcll(ballot(mn < t));
#endif
        if constexpr (kHier) {
          // the regions whose view changes in this round (one advert per due lane): only
          // their cached regional minima are dropped
          const int gd = mn < t ? mj / (kWave * kWideGroupSlots) : -1;
          uint64_t m = ballot(gd >= 0);
          while (m) {
            const int rg = __builtin_amdgcn_readlane(gd, (int)__builtin_ctzll(m));
            reg_dirty |= 1ull << rg;
            m &= ~ballot(gd == rg);
          }
        }
        if (mn < t) {
          const int j = mj;
          const int sl = j / kWave;
          int64_t nxt_j;
          uint32_t busy_j;
          const bool hit = j == cj;
          const int g = sl / kWideGroupSlots;
          const int si = sl % kWideGroupSlots;
          // node j's adverts that are due: adverts of different nodes commute (each sets only
          // its node's view), so j's later due ones are applied now, in their order, and only
          // the last one's view is stored and rescanned (no store between the dependent entry
          // loads).  The cached record is updated in place (no copy through a merged value).
          bool broken = false, fits = true;
          int64_t w_j = kNever;
          auto apply_due = [&](WideNode& hh, int64_t dl, int64_t ul) {
            fits = apply_wide_advert(hh, e, dl, ul, kHier ? A.hier_up : 0, nxt_j, busy_j, broken, PF_WALK);
            while (nxt_j < t && !broken) {
#ifdef FOGNET_WIDE_PROF
              ++pf_same;
#endif
              fits &= apply_wide_advert(hh, e, dl, ul, kHier ? A.hier_up : 0, nxt_j, busy_j, broken, PF_WALK);
            }
            if constexpr (!kPerPublish) w_j = node_w(hh, nxt_j, dl);
          };
          if (hit) {
            apply_due(ch, c_dl, c_ul);
          } else {  // (waited for in this arm: sync_vm)
            WideNode h = nd[j];
            const int64_t dl_j = P_dl[j], ul_j = P_ul[j];
            sync_vm();
            apply_due(h, dl_j, ul_j);
            nd[j] = h;
          }
          if constexpr (kExt) lerr |= !fits;
          lbroken |= broken;
          V.nxt[sl] = nxt_j;
          V.busy[sl] = busy_j;
          // the earliest advert: j's was the lane's (so its group's), rescan both levels, the
          // group over its other pending slots only (ties: the smallest slot)
          const uint32_t gm0 = L.g_msk[g * kWave + lane];
          const uint32_t bit = 1u << si;
          uint32_t gm = nxt_j != kNever ? gm0 | bit : gm0 & ~bit;
          gm = busy_j != 0u ? gm | (bit << 16) : gm & ~(bit << 16);
          L.g_msk[g * kWave + lane] = gm;
          int64_t gmn = nxt_j, gmw = w_j;
          int gsi = si;
          if constexpr (!kPerPublish) V.w[sl] = w_j;
          // the group's other pending slots, four at a time: their view loads are all issued before
          // the first compare (one HBM round trip per four slots, not per slot)
          for (uint32_t m = gm0 & 0xFFFFu & ~bit; m;) {
            int ix[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              ok[u] = m != 0u;
              ix[u] = ok[u] ? __builtin_ctz(m) : 0;
              m = ok[u] ? m & (m - 1u) : m;
            }
            int64_t xs[4], ws[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              xs[u] = V.nxt[g * kWideGroupSlots + ix[u]];
              ws[u] = kNever;
              if constexpr (!kPerPublish) ws[u] = V.w[g * kWideGroupSlots + ix[u]];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (!ok[u]) continue;
              if (xs[u] < gmn || (xs[u] == gmn && ix[u] < gsi)) {
                gmn = xs[u];
                gsi = ix[u];
              }
              gmw = ws[u] < gmw ? ws[u] : gmw;
            }
          }
          L.g_nxt[g * kWave + lane] = gmn;
          L.g_j[g * kWave + lane] = gmn == kNever ? lane : wnode<kHier>(g * kWideGroupSlots + gsi, lane);
          gact.set(g, (gm & 0xFFFFu) != 0u);
          if constexpr (!kPerPublish) {
            L.g_w[g * kWave + lane] = gmw;
            lane_min_nxt_w_m(L, lane, gact, mn, mj, mw);  // (one LDS pass for both lane minima)
          } else {
            lane_min_nxt_m(L, lane, gact, mn, mj);
          }
#ifdef FOGNET_WIDE_PROF
          pf_hit += hit ? 1u : 0u;
#endif
          // the view key: only j's changed; the group (and lane) minimum needs a rescan only
          // when j held it and its busy time grew
          const uint64_t gk_old = L.g_key[g * kWave + lane];
          const uint64_t nk = ((uint64_t)busy_j << 32) | (uint32_t)j;
          const uint64_t gk_new = ((uint32_t)gk_old == (uint32_t)j && nk > gk_old) ? group_key_m<kHier>(V, L, lane, g)
                                                                                 : (nk < gk_old ? nk : gk_old);
#ifdef FOGNET_WIDE_PROF
          pf_gkey += ((uint32_t)gk_old == (uint32_t)j && nk > gk_old) ? 1u : 0u;
#endif
          L.g_key[g * kWave + lane] = gk_new;
          if (gk_new < mk) mk = gk_new;
          else if (mk == gk_old && gk_new > gk_old) mk = lane_min_key(L, lane);
        }
      }
      if (ballot(lbroken)) {
        err = FOGNET_ERR_INTERNAL;
        break;
      }
      if (ballot(lerr)) {
        err = FOGNET_ERR_CAPACITY;
        break;
      }

      WTM(1)
      // 2) the decision over the advertised view
      bool escalated = false;
      if constexpr (kExt) {
        // north-star cost (fognet_hip.h FOGNET_POLICY_EXT_LAT), first index on ties; per publish
        const uint32_t rq = readlane_u32((uint32_t)cr, jp);
        uint64_t mc = ~0ull;
        uint32_t mjj = ~0u;
        for (int sj = 0; sj < SP; ++sj) {  // this lane's nodes (its view)
          const int j = wnode<kHier>(sj, lane);
          if (j >= N) continue;
          const uint32_t S = min(rq / (uint32_t)P_mips[j], kExtSatS);
          const uint64_t c = (uint64_t)P_dl[j] + ((uint64_t)V.busy[sj] + S) * (uint64_t)kTicksPerSecond;
          if (c < mc) {
            mc = c;
            mjj = (uint32_t)j;
          }
        }
        const uint64_t m = wave_min_u64(mc);
        k = wave_min_u32(mc == m ? mjj : ~0u);
      } else if constexpr (kHier) {
        // regional broker: the smallest (busy, index) of its region (the region's LDS group
        // minima, one per lane); above the threshold the parent takes the global one.  Both
        // are kept until an advert changes the view (the LDS region cache, bit b of reg_valid).
        const int b = __builtin_amdgcn_readlane(cg, jp);
        if (view_changed) {
          reg_valid &= ~reg_dirty;
          reg_dirty = 0ull;
          glob_valid = false;
          view_changed = false;
        }
        uint64_t kb;
        if ((reg_valid >> b) & 1ull) {
          kb = L.reg_key[b];
        } else {
          kb = wave_min_u64(L.g_key[b * kWave + lane]);
          if (lane == 0) L.reg_key[b] = kb;
          reg_valid |= 1ull << b;
        }
        escalated = (kb >> 32) > (uint64_t)A.hier_thr;
        if (escalated && !glob_valid) {
          glob_key = wave_min_u64(mk);
          glob_valid = true;
        }
        if (((escalated ? glob_key : kb) >> 32) >= kBusySat) {  // the minimum is past 32 bits
          err = FOGNET_ERR_CAPACITY;
          break;
        }
        k = escalated ? (uint32_t)glob_key : (uint32_t)kb;
      } else if (view_changed) {
        // BrokerBaseApp3.cc:267-281: busy_j + req/mips_0 < tempp over exact
        // integer busy values <=> the smallest (busy, j)
        k_key = wave_min_u64(mk);
        k = (uint32_t)k_key;
        view_changed = false;
        if ((k_key >> 32) >= kBusySat) {  // the minimum is past 32 bits: exact order unknown
          err = FOGNET_ERR_CAPACITY;
          break;
        }
      }
      const int kl = wlane<kHier>((int)k);

      WTM(2)
      // 3) node k's record and parameters, in its owner lane (cached there)
      cache_node(k);
      uint32_t pend_k = 0u;  // EXT_HIER: k's escalated tasks still pending (decided, not pushed)
      if constexpr (kHier) {
        if (escalated) {  // wait in a pending slot until the tasks that reach k before it are pushed
          const uint64_t fr = n_ovf ? 0ull : ballot(L.p_i[lane] < 0);
          const int64_t a_esc = t + readlane_i64(c_dl, kl) + A.hier_up;
          const uint32_t rq = readlane_u32((uint32_t)cr, jp);
          if (fr) {
            const int sl = (int)__builtin_ctzll(fr);
            if (lane == sl) {
              L.p_i[lane] = c0 + jp;
              L.p_t[lane] = t;
              L.p_a[lane] = a_esc;
              L.p_k[lane] = (int32_t)k;
              L.p_r[lane] = rq;
            }
          } else {  // all slots taken (or the list in use): the overflow list in HBM
            if (lane == 0) {
              e[c0 + jp] = WideEntry{a_esc, t, 0u, rq, (int32_t)k, -1, 2};
              ov[ov_tail] = c0 + jp;
            }
            ++ov_tail;
            ++n_ovf;
          }
          ++n_pend;
          const uint32_t tot = (uint32_t)readlane_u32((uint32_t)ch.npend, kl) + pend_count(k);
          max_pend = max(max_pend, tot);
          n_done += 1;
          jp += 1;
          WTM(3)  // (profile builds: the escalation's pending bookkeeping counts as "record")
          continue;
        }
        // a direct task: the pending escalated tasks that reach k no later than it go first
        if (n_pend) {
          if (!flush_pending(true, k, t + readlane_i64(c_dl, kl))) {
            err = FOGNET_ERR_ARG;
            break;
          }
          cache_node(k);
          pend_k = pend_count(k);  // (those it overtakes)
        }
      }
      const int32_t mips_k = (int32_t)readlane_u32((uint32_t)c_mips, kl);
      const UDiv div_k{readlane_u32((uint32_t)c_dv, kl), readlane_u32((uint32_t)(c_dv >> 32), kl)};
      // (an escalated task takes the regional -> parent hop before the downlink)
      const int64_t dl_k = readlane_i64(c_dl, kl) + (escalated ? A.hier_up : 0);
      const int64_t ul_k = readlane_i64(c_ul, kl), down_k = readlane_i64(c_down, kl);
      const int32_t tl = (int32_t)readlane_u32((uint32_t)ch.tl, kl);
      const int32_t npend0 = (int32_t)readlane_u32((uint32_t)ch.npend, kl);
      const int64_t tl_done = readlane_i64(ch.tl_done, kl);
      const uint64_t tl_C = (uint64_t)readlane_i64((int64_t)ch.tl_C, kl);
      const uint32_t tl_S = readlane_u32(ch.tl_S, kl) & 0x7FFFFFFFu;  // (bit 31: the tail was escalated)
      const int64_t base_done = tl >= 0 ? tl_done : INT64_MIN;  // kNever: the node crashed with work left

      WTM(3)
      // 4) the run: publishes jp .. jq-1 up to the earliest pending advert E
      //    (an advert of any node may change the view) all go to node k; when
      //    k has nothing pending, the run's first task becomes its head and
      //    that task's advert bounds the run too
      int jq = jp + 1;
      if constexpr (!kPerPublish) {
        // run horizon (node_w), per group of the lane with a pending advert: node j takes the
        // decision from k = (busy_b, k) only with an advert of busy v <= thr_j = busy_b - (j > k)
        // (ties -> the lower index), which comes no earlier than max(nxt_j, w_j - thr_j s), so
        // the group's adverts none before max(min nxt, min w - thr s) with thr its largest thr_j;
        // a group whose nodes all have larger indices than k, with busy_b = 0, never matters
        const uint32_t busy_b = (uint32_t)(k_key >> 32);
        int64_t e_lane = kNever;
        gact.each([&](int g) {
          const uint32_t thr = busy_b - (((uint32_t)(g * kWave * kWideGroupSlots) + (uint32_t)lane > k) ? 1u : 0u);
          if (thr == 0xFFFFFFFFu) return;  // (busy_b = 0 and every node of the group after k)
          const int64_t gx = L.g_nxt[g * kWave + lane], gw = L.g_w[g * kWave + lane];
          int64_t bnd = gx;
          if (thr < (1u << 21) && (uint64_t)(gw - gx) > (uint64_t)ticks_of(thr)) bnd = gw - ticks_of(thr);
          e_lane = bnd < e_lane ? bnd : e_lane;
        });
        int64_t E = (int64_t)wave_min_u64((uint64_t)e_lane);
        if (npend0 > 0) {  // k's own next advert changes its key
          const int64_t hd_done_k = readlane_i64(ch.hd_done, kl);
          const int64_t nxt_k = hd_done_k == kNever ? kNever : hd_done_k + ul_k;
          E = nxt_k < E ? nxt_k : E;
        }
        if (npend0 == 0) {
          const uint32_t S0 = readlane_u32((uint32_t)cr, jp) / (uint32_t)mips_k;
          const int64_t a0 = t + dl_k;
          int64_t x0 = kNever;
          if (a0 < down_k && base_done != kNever) {
            const int64_t st0 = a0 > base_done ? a0 : base_done;
            const int64_t d0 = st0 + ticks_of(min(S0, kWideSCap));
            if (st0 < down_k && d0 < down_k) x0 = d0 + ul_k;
          }
          E = x0 < E ? x0 : E;
        }
        const uint64_t run_mask = ballot((lane >= jp && lane < cnt && ca <= E) || lane == jp);
        // the run is the contiguous lanes from jp (ticks are nondecreasing)
        jq = jp + __popcll(run_mask >> jp);
      }
      const bool in_run = lane >= jp && lane < jq;
      const int Lr = jq - jp;
#ifdef FOGNET_WIDE_PROF
      ++pf_runs;
#endif

      // 5) task arrivals at node k (ComputeBrokerApp3.cc:269-320), one lane per
      //    task: FIFO single server, done_m = max(a_m, done_{m-1}) + S_m
      uint32_t S = 0u;
      int64_t a = 0;
      bool lerr2 = false;
      if (in_run) {
        S = udiv((uint32_t)cr, div_k);  // double tskTime = requiredMIPS / MIPS (:276)
        a = ca + dl_k;
      }
      const uint32_t Sd = min(S, kWideSCap);  // tick arithmetic (kWideSCap)
      const bool one = Lr == 1;               // a single publish needs no wave scans
      // service seconds of the run up to this task: clamped for the ticks (<= 64 * 2^22 < 2^32),
      // exact in 64 bits for the cumulative service (a run with a longer service time is rare)
      const uint32_t Cs = one ? (in_run ? Sd : 0u) : wave_scan_add_u32(in_run ? Sd : 0u);
      uint64_t Cs64 = Cs;
      if (ballot(in_run && S >= kWideSCap))
        Cs64 = one ? (uint64_t)(in_run ? S : 0u) : (uint64_t)wave_scan_add_i64(in_run ? (int64_t)S : 0);
      const uint64_t C = tl_C + Cs64;  // cumulative assigned service
      int64_t start = kNever, done = kNever;
      uint32_t status = FOGNET_TASK_LOST;
      if (base_done != kNever) {
        int64_t X = in_run ? (int64_t)((uint64_t)a - (uint64_t)ticks_of(min(Cs - Sd, kWideSCap))) : INT64_MIN;
        if (!one) X = wave_scan_max_i64(X);
        const int64_t dmax = base_done > X ? base_done : X;
        // start = dmax + the run's service before the task, done = dmax + through it; a prefix of
        // 2^22 s or more puts the tick past kMaxTick (kPastRange: lost to a crash, else refused below;
        // a clamped X only over-estimates lanes whose own prefix is past the cap)
        const int64_t st = Cs - Sd < kWideSCap ? dmax + ticks_of(Cs - Sd) : kPastRange;
        const int64_t dn = Cs < kWideSCap ? dmax + ticks_of(Cs) : kPastRange;
        int64_t prev_done = base_done;
        uint32_t prev_S = tl_S;
        if (!one) {
          const int64_t dn_up = dpp_or_i64<kDppWaveShr1>(0, dn);
          const uint32_t S_up = dpp_or_u32<kDppWaveShr1>(0u, Sd);
          if (lane != jp) {
            prev_done = dn_up;
            prev_S = S_up;
          }
        }
        if (in_run && a < down_k) {
          if (prev_done < a) status = 5u;       // idle: "task assigned" (:282-301)
          else if (prev_done > a) status = 4u;  // busy: "task queued" (:304-313)
          else status = dl_k < (int64_t)min(prev_S, kWideSCap) * kTicksPerSecond ? 5u : 4u;  // same-tick completion
          start = st < down_k ? st : kNever;   // the crash cancels its RELEASERESOURCE
          done = dn < down_k ? dn : kNever;
        }
      } else if (in_run && a < down_k) {
        status = 4u;  // queued behind a task the crashed node never completes
      }
      lerr2 = in_run && (a > kMaxTick || (done != kNever && done > kMaxTick));
      if (ballot(lerr2)) {
        err = FOGNET_ERR_ARG;
        break;
      }
      // task entries: chained in publish order (consecutive task indices)
      const int i = c0 + lane;
      if (in_run) {
        const int32_t prev = lane == jp ? tl : i - 1;
        e[i] = WideEntry{a, done, C, S, prev, lane + 1 < jq ? i + 1 : -1, escalated ? 1 : 0};
        q_on = true;
        q_k = k;
        q_a = a;
        q_start = start;
        q_done = done;
        q_S = S;
        q_status = status;
      }

      WTM(4)
      // 6) node k's record after the run (owner lane)
      const int lz = jq - 1;
      const int64_t a_z = readlane_i64(a, lz), done_z = readlane_i64(done, lz);
      const uint64_t C_z = (uint64_t)readlane_i64((int64_t)C, lz);
      const uint32_t S_z = readlane_u32(S, lz);
      const int64_t done_f = readlane_i64(done, jp);
      const uint64_t C_f = (uint64_t)readlane_i64((int64_t)C, jp);
      const uint32_t S_f = readlane_u32(S, jp);
      if (lane == kl) {
        WideNode h = ch;
        const int i0 = c0 + jp, iz = c0 + lz;
        if (h.npend == 0) {  // the run's first task is the node's head: its advert is the node's next one
          h.hd = i0;
          h.hd_done = done_f;
          h.hd_C = C_f;
          h.hd_S = S_f;
          const int64_t x = done_f == kNever ? kNever : done_f + ul_k;
          const int g = ((int)k / kWave) / kWideGroupSlots;
          V.nxt[k / kWave] = x;
          if (x != kNever) {
            L.g_msk[g * kWave + lane] |= 1u << ((k / kWave) % kWideGroupSlots);
            gact.set(g, true);
          }
          if (x < L.g_nxt[g * kWave + lane]) {
            L.g_nxt[g * kWave + lane] = x;
            L.g_j[g * kWave + lane] = (int)k;
          }
          if (x < mn) {
            mn = x;
            mj = (int)k;
          }
        } else if (h.npend >= 2) {
          e[h.tl].next = i0;
        }
        // hd_next after the two-way branch, not in a third arm (DESIGN.md §3.6 "The hd_next
        // miscompile"): the run's second task on an idle node, its first on a node whose one
        // pending task is the tail
        if (h.npend == 1 || (h.npend == 0 && Lr > 1)) h.hd_next = h.npend == 1 ? i0 : i0 + 1;
        h.tl = iz;
        h.tl_a = a_z;
        h.tl_done = done_z;
        h.tl_C = C_z;
        h.tl_S = S_z | (escalated ? 0x80000000u : 0u);
        h.npend += Lr;
        ch = h;
        max_pend = max(max_pend, (uint32_t)h.npend + pend_k);
        if constexpr (!kPerPublish) {
          // k's w (a larger value may leave its group minimum stale-small: conservative)
          const int sk = (int)k / kWave, gk = sk / kWideGroupSlots;
          const int64_t nxt_k = h.hd_done == kNever ? kNever : h.hd_done + ul_k;
          const int64_t w_k = node_w(h, nxt_k, c_dl);
          V.w[sk] = w_k;
          if (w_k < L.g_w[gk * kWave + lane]) L.g_w[gk * kWave + lane] = w_k;
          if (w_k < mw) mw = w_k;
        }
      }
      n_done += Lr;
      WTM(5)
      jp = jq;
    }
    WTM(0)
    // the chunk's outputs and statistics (also after an error ended it: the tasks pushed so far)
    if (q_on && !A.no_task_out) {  // (statistics-only replays keep no per-task outputs)
      const size_t o = tbase + (size_t)(c0 + lane);
      A.out_node[o] = (int32_t)q_k;
      A.out_status[o] = (uint8_t)q_status;
      A.out_start[o] = q_start == kNever ? -1 : q_start;
      A.out_done[o] = q_done == kNever ? -1 : q_done;
    }
    if (q_on) {
      if (q_done != kNever) {
        acc_task(acc, ab, ca, q_a, q_start, q_done, q_S, q_status, c0 + lane, hist ? L.hist : nullptr);
        if (hist) atomicAdd(&L.hist[FOGNET_HIST_BINS + hist_bin(q_done - ca)], 1u);
      } else {
        // node-down: acked at arrival (status 4/5) or lost; a queued task that
        // started before the crash still emitted its queueTime (:238)
        n_short += 1;
        if (q_status == 5u) acc.n5 += 1u;
        if (q_status == 4u) {
          acc.n4 += 1u;
          if (q_start != kNever) acc_qtime(acc, ab, q_start, q_a, c0 + lane, hist ? L.hist : nullptr);
        }
      }
    }
  }

  if constexpr (kHier) {  // the escalated tasks still in flight at the end, then their statistics
    if (err == FOGNET_OK && n_pend && !flush_pending(false, 0u, INT64_MAX)) err = FOGNET_ERR_ARG;
    if (n_sq) drain_stats();
  }
  if (cj >= 0) nd[cj] = ch;

  // ---- per-replication record (the fields replay_kernel + its epilogue write)
#ifdef FOGNET_WIDE_PROF
  for (int m = kWave / 2; m > 0; m >>= 1) {
    pf_same += shfl_xor_u64(pf_same, m);
    pf_hit += shfl_xor_u64(pf_hit, m);
    pf_gkey += shfl_xor_u64(pf_gkey, m);
  }
  const uint64_t pf_w1 = wave_sum_u64((uint64_t)(pf_walk & 0xFFFFu)), pf_w2 = wave_sum_u64((uint64_t)(pf_walk >> 16));
#endif
  acc = wave_merge(acc);
  ab = wave_min_abort(ab);
  const uint32_t mp = ~wave_min_u32(~max_pend);
  int shorts = n_short;
  for (int m = kWave / 2; m > 0; m >>= 1) shorts += __shfl_xor(shorts, m, kWave);
  fognet_rep_stats* const S = A.out_stats + r;
  if (lane == 0 && A.out_stats) {
    S->n_tasks = n_done;
    S->max_pending = (int32_t)mp;
    S->status = (int32_t)err;
    // initial adverts + publish, arrival, release, advert per task (publish,
    // arrival for a task a crash keeps from completing)
    S->events = 2 * (int64_t)N + 4 * (int64_t)n_done - 2 * (int64_t)shorts;
    write_rep_stats(S, acc, ab, A.ref_abort);
#ifdef FOGNET_WIDE_PROF
    S->queue_sum_lo = pf_iter;
    S->queue_sum_hi = pf_advit;
    S->queue_sq_lo = pf_adv;
    S->resp_sum_lo = pf_runs;
    S->resp_sum_hi = pf_same;
    S->resp_sq_lo = pf_hit;
    S->resp_sq_hi = pf_gkey;
    S->queue_min_raw = (int64_t)pf_t[0];  // chunk end: outputs + statistics
    S->queue_max_raw = (int64_t)pf_t[1];  // adverts (incl. flush of pending escalations)
    S->resp_min_ticks = (int64_t)pf_t[2]; // decision
    S->resp_max_ticks = (int64_t)pf_t[3]; // record + parameters (+ EXT_HIER escalation handling)
    S->last_tick = (int64_t)pf_t[4];      // run horizon + FIFO + entries
    S->queue_sq_top = pf_t[5];            // record update
    S->busy_s = (int64_t)pf_t[6];         // chunk start: trace load + preconditions
    S->n_started = (int64_t)(pf_w1 | (pf_w2 << 32));  // walks | steps << 32
#endif
  }
  // a11 energy (fognet_hip.h): E_j = P_busy_j * B_j + P_idle_j * ((H - B_j 1e12) / 1e12)
  // with B_j = node j's service seconds (its tail's cumulative sum), summed in node order
  if (A.p_busy && A.out_stats) {
    __syncthreads();  // (the records written back above by their owner lanes are read by others)
    // per node j (lane j % 64 here), then summed in node order 64 at a time
    const int64_t H = n_done > 0 ? acc.last : 0;
    static_assert(sizeof(WideNode) % sizeof(uint64_t) == 0 && offsetof(WideNode, tl_C) % sizeof(uint64_t) == 0, "tl_C stride");
    const double sum = energy_sum_wave(reinterpret_cast<const uint64_t*>(reinterpret_cast<const char*>(nd) + offsetof(WideNode, tl_C)),
                                       (int)(sizeof(WideNode) / sizeof(uint64_t)), A.p_busy + nbase, A.p_idle + nbase, N, H,
                                       A.out_energy ? A.out_energy + (size_t)r * (size_t)N : nullptr, lane,
                                       // (LDS the loop no longer reads: the group minima or, BIG, the group mask words)
                                       reinterpret_cast<double*>(BIG ? reinterpret_cast<unsigned char*>(gw_lds) : w_lds));
    if (lane == 0) S->energy_j = sum;
  }
  if (hist) {
    __syncthreads();
    for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave)
      if (L.hist[h]) atomicAdd((unsigned long long*)&A.hist[h], (unsigned long long)L.hist[h]);
  }
}

template <int POL, bool BIG>
void launch_wide_pol(const ReplayArgs& a, int32_t slots, WideEntry* e, WideNode* nd, int64_t* vn, uint32_t* vb,
                     int64_t* vw, GenNodes gn, int32_t* ov, unsigned char* gx, const RegionWs& rw, size_t lds,
                     hipStream_t s) {
  if (lds > 65536)  // above the default dynamic-LDS limit (N > ~51,000 nodes; gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&replay_wide_kernel<POL, BIG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL((replay_wide_kernel<POL, BIG>), dim3(slots), dim3(kWave), lds, s, a, e, nd, vn, vb, vw, gn, ov,
                     gx, rw);
}

// FOGNET_WIDE_BIG=1: the HBM group minima at any N (the flat policies; parity tests of both layouts)
bool wide_force_big() {
  const char* f = getenv("FOGNET_WIDE_BIG");
  return f && f[0] == '1';
}


// (big: wide_big -- the group minima in HBM, the active-group mask words in LDS)
size_t wide_lds_bytes(int32_t N, bool big) {
  const size_t G = (size_t)wide_groups(N);
  const size_t rest = FOGNET_HIST_METRICS * FOGNET_HIST_BINS * sizeof(uint32_t) +
                      kHierPending * (2 * sizeof(int64_t) + 3 * sizeof(int32_t)) +
                      kWave * (4 * sizeof(int64_t) + 2 * sizeof(int32_t));
  if (big) return rest + (size_t)kGWords * kWave * sizeof(uint64_t);
  return G * kWave * (sizeof(int64_t) + sizeof(uint64_t) + sizeof(int64_t) + sizeof(int32_t)) + rest +
         G * sizeof(uint64_t) + G * kWave * sizeof(uint32_t);
}

}  // namespace

size_t replay_wide_lds_bytes(int32_t N) { return wide_lds_bytes(N, wide_big(N, false)); }

// (the EXT_HIER regions stay groups in LDS: N <= kWideMaxNodes, never BIG)
static bool wide_big_for(int32_t N, int policy) {
  return policy != FOGNET_POLICY_EXT_HIER && wide_big(N, wide_force_big());
}

size_t replay_wide_workspace_bytes(int32_t R, int32_t T, int32_t N, bool gen, int policy) {
  return wide_ws(R, T, N, gen, wide_big_for(N, policy)).bytes;
}

hipError_t launch_replay_wide(const ReplayArgs& a, void* workspace, int32_t slots, hipStream_t s, const RegionWs* rwp) {
  RegionWs rw{};  // (esc null: every listed replication starts from the beginning)
  if (rwp && a.policy == FOGNET_POLICY_EXT_HIER) rw = *rwp;
  const bool big = wide_big_for(a.N, a.policy);
  const WideWs w = wide_ws(slots, a.T, a.N, a.gen_on != 0, big);
  unsigned char* const base = static_cast<unsigned char*>(workspace);
  WideEntry* const e = reinterpret_cast<WideEntry*>(base + w.e_off);
  WideNode* const nd = reinterpret_cast<WideNode*>(base + w.nd_off);
  int64_t* const vn = reinterpret_cast<int64_t*>(base + w.nxt_off);
  uint32_t* const vb = reinterpret_cast<uint32_t*>(base + w.busy_off);
  int64_t* const vw = reinterpret_cast<int64_t*>(base + w.w_off);
  const GenNodes gn{reinterpret_cast<int32_t*>(base + w.gm_off), reinterpret_cast<int64_t*>(base + w.gd_off),
                    reinterpret_cast<int64_t*>(base + w.gu_off), reinterpret_cast<uint64_t*>(base + w.dv_off)};
  int32_t* const ov = reinterpret_cast<int32_t*>(base + w.ov_off);
  unsigned char* const gx = base + w.gx_off;
  const size_t lds = wide_lds_bytes(a.N, big);
  if (a.policy == FOGNET_POLICY_EXT_LAT) {
    if (big)
      launch_wide_pol<FOGNET_POLICY_EXT_LAT, true>(a, slots, e, nd, vn, vb, vw, gn, ov, gx, rw, lds, s);
    else
      launch_wide_pol<FOGNET_POLICY_EXT_LAT, false>(a, slots, e, nd, vn, vb, vw, gn, ov, gx, rw, lds, s);
  } else if (a.policy == FOGNET_POLICY_EXT_HIER) {
    launch_wide_pol<FOGNET_POLICY_EXT_HIER, false>(a, slots, e, nd, vn, vb, vw, gn, ov, gx, rw, lds, s);
  } else if (big) {
    launch_wide_pol<FOGNET_POLICY_REF_V3, true>(a, slots, e, nd, vn, vb, vw, gn, ov, gx, rw, lds, s);
  } else {
    launch_wide_pol<FOGNET_POLICY_REF_V3, false>(a, slots, e, nd, vn, vb, vw, gn, ov, gx, rw, lds, s);
  }
  return hipGetLastError();
}

}  // namespace fognet
