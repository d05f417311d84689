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
// closed form:
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
//
// Decision runs.  The broker's view is stale, so consecutive publishes keep
// going to the same node until an advert changes the argmin (runs of 50-200
// publishes at the C3 sweep).  The kernel finds, lane-parallel, the earliest
// advert that could change the decision (run horizon), then pushes the whole
// run (up to the 64 publishes of a trace chunk, one per lane) with a (max,+)
// scan over the FIFO recurrence and coalesced ring and output stores.
#include "replay_common.h"

namespace fognet {

namespace {

struct Slot {
  uint32_t vkey;     // broker view of the node: (advertised busy seconds << 8) | node index
  int64_t nxt;       // tick at which the head's completion advert reaches the broker
  // (head completion tick = nxt - ul: the advert leaves the node at completion)
  uint32_t hd_C;     // cumulative service up to and including the head
  uint32_t hd_S;     // head service seconds (< 2^24)
  // (the 16-B ring pair holding entry head+1 lives in reserved VGPRs, see
  //  nh_prefetch; RingWord layout in internal.h)
  int64_t tl_a;      // tail (newest) task: arrival tick at the node
  // (tail completion tick, cumulative service and service time live in LDS:
  //  s_tld / s_tlC / s_tlS, read at a uniform address when the node is chosen)
  uint32_t cnt;      // ring counters mod 2^16: tasks ever assigned (bits 0-15),
                     // completion adverts applied (bits 16-31); capacity <= 2^15
};

// Profile builds (`make prof`, tools/replay_counters.py) only:
// FOGNET_REPLAY_PROFILE=1 counts loop events, =2 accumulates s_memtime cycles
// per loop segment; either is written into the stats record.
#if FOGNET_REPLAY_PROFILE == 1
#define PROF(x) x
#else
#define PROF(x)
#endif
#if FOGNET_REPLAY_PROFILE == 2
#define TMARK(i)                                            \
  {                                                         \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();     \
    p_t[i] += now_ - p_last;                                \
    p_last = now_;                                          \
  }
#else
#define TMARK(i)
#endif

constexpr uint32_t kNoKey = ~0u;

__device__ __forceinline__ uint32_t n_push(const Slot& st) { return st.cnt & 0xFFFFu; }
__device__ __forceinline__ uint32_t n_head(const Slot& st) { return st.cnt >> 16; }
__device__ __forceinline__ uint32_t pending(const Slot& st) { return (n_push(st) - n_head(st)) & 0xFFFFu; }
__device__ __forceinline__ uint32_t head_S(const Slot& st) { return st.hd_S; }
// Ring pairs: entries 2p and 2p + 1 of a node's ring share one 16-B aligned
// pair; the reserved registers of a slot hold the pair of its head+1 entry.
// Entry head+1 is its odd half when head+1 is odd.
__device__ __forceinline__ uint32_t nh_odd(const Slot& st) { return (n_head(st) + 1u) & 1u; }
__device__ __forceinline__ RingWord nh_word(u32x4 v, uint32_t odd) {
  return odd ? (((uint64_t)v.w << 32) | v.z) : (((uint64_t)v.y << 32) | v.x);
}
__device__ __forceinline__ int64_t rw_a(RingWord w) { return (int64_t)(w >> kRingSBits); }
__device__ __forceinline__ uint32_t rw_S(RingWord w) { return (uint32_t)w & kRingSMask; }

// ---- head+1 prefetch, outside the compiler's register allocation
//
// The head+1 entry of a node is needed at that node's next advert, typically
// many publishes later.  A compiler-visible load cannot express that: its
// loop-carried destination gets a conservative `s_waitcnt vmcnt(0)` at the
// first read in the next loop iteration (loads and stores share the in-order
// vmcnt counter, and the count between issue and use is data dependent), and
// a value the compiler believes is ready may be copied between registers
// while the load is still in flight.  So the entries live in VGPRs the
// compiler never allocates: the kernel caps allocation at kNhBase
// (amdgpu_num_vgpr; on gfx90a+ the attribute counts half the unified
// register file, so kNhBase / 2) and slot s of every lane owns v[kNhBase + 4s .. +3].  Only
// inline asm names them: the prefetch loads, and nh_read, which waits and
// copies them out in one statement (tools/check_nh_regs.py audits the ISA).
//
// The wait count comes from a wave-uniform tally `ops` of vector-memory
// instructions that are certainly issued (the chunk loads, the five stores of
// every push run, slot refills and advert prefetches).  A node's prefetch is
// stamped with the tally including itself; `ops - stamp` tallied
// instructions were issued after it, so `s_waitcnt vmcnt(ops - stamp)`
// (capped at kPrefetchOps) covers it.  Untallied instructions only make the
// real count larger (safe).  The stamp keeps 8 bits; a wrapped stamp can only
// make an old prefetch look recent.  Vector-memory operations complete in
// issue order for vmcnt, so the newest prefetch into a register wins.
constexpr uint32_t kPrefetchOps = 8;
constexpr int kNhBase = 112;  // v112..v127: 4 slots x {a lo, a hi, C, S}
static_assert(kNhBase + 4 * kMaxNodesPerLane == 128, "4 waves/SIMD: 128 VGPRs per lane");
// Generated mode (replay_gen_kernel) keeps the statistics accumulators in
// registers through the loop: 3 waves/SIMD, allocation capped at 152, the
// prefetch registers are v152..v167 (register set 1: slot functions 4..7).
constexpr int kNhBaseGen = 152;
static_assert(kNhBaseGen + 4 * kMaxNodesPerLane == 168, "3 waves/SIMD: 168 VGPRs per lane");

#define FOGNET_NH_SLOT(S, R0, R1, R2, R3, RR)                                                  \
  __device__ __forceinline__ void nh_prefetch_##S(const RingWord* p) {                       \
    asm volatile("global_load_dwordx4 " RR ", %0, off" : : "v"(p) : "memory", R0, R1, R2, R3); \
  }                                                                                           \
  /* one lane's load: EXEC narrowed inside the statement (uniform control flow) */           \
  __device__ __forceinline__ void nh_refill_##S(const RingWord* p, uint64_t only) {          \
    uint64_t saved;                                                                           \
    asm volatile("s_mov_b64 %0, exec\n\t"                                                     \
                 "s_mov_b64 exec, %2\n\t"                                                     \
                 "global_load_dwordx4 " RR ", %1, off\n\t"                                    \
                 "s_mov_b64 exec, %0"                                                         \
                 : "=&s"(saved)                                                               \
                 : "v"(p), "s"(only)                                                          \
                 : "memory", R0, R1, R2, R3);                                                 \
  }                                                                                           \
  /* wait until at most m vector-memory instructions are outstanding (s_waitcnt  */          \
  /* takes an immediate: branch to the right one; m >= 8 -> vmcnt(8)), then copy */          \
  __device__ __forceinline__ u32x4 nh_read_##S(uint32_t m) {                                  \
    uint32_t x, y, z, w;                                                                      \
    asm volatile(                                                                             \
      "s_cmp_lt_u32 %4, 8\n\t"                                                                 \
      "s_cbranch_scc1 1f\n\t"                                                                   \
      "s_waitcnt vmcnt(8)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "1:\n\t"                                                                                  \
      "s_cmp_lt_u32 %4, 6\n\t"                                                                  \
      "s_cbranch_scc1 2f\n\t"                                                                   \
      "s_cmp_eq_u32 %4, 6\n\t"                                                                  \
      "s_cbranch_scc1 3f\n\t"                                                                   \
      "s_waitcnt vmcnt(7)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "3:\n\t"                                                                                  \
      "s_waitcnt vmcnt(6)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "2:\n\t"                                                                                  \
      "s_cmp_lt_u32 %4, 4\n\t"                                                                  \
      "s_cbranch_scc1 4f\n\t"                                                                   \
      "s_cmp_eq_u32 %4, 4\n\t"                                                                  \
      "s_cbranch_scc1 5f\n\t"                                                                   \
      "s_waitcnt vmcnt(5)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "5:\n\t"                                                                                  \
      "s_waitcnt vmcnt(4)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "4:\n\t"                                                                                  \
      "s_cmp_lt_u32 %4, 2\n\t"                                                                  \
      "s_cbranch_scc1 6f\n\t"                                                                   \
      "s_cmp_eq_u32 %4, 2\n\t"                                                                  \
      "s_cbranch_scc1 7f\n\t"                                                                   \
      "s_waitcnt vmcnt(3)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "7:\n\t"                                                                                  \
      "s_waitcnt vmcnt(2)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "6:\n\t"                                                                                  \
      "s_cmp_eq_u32 %4, 1\n\t"                                                                  \
      "s_cbranch_scc0 8f\n\t"                                                                   \
      "s_waitcnt vmcnt(1)\n\t"                                                                  \
      "s_branch 9f\n"                                                                           \
      "8:\n\t"                                                                                  \
      "s_waitcnt vmcnt(0)\n"                                                                    \
      "9:\n\t"                                                                                  \
      "v_mov_b32 %0, " R0 "\n\t"                                                                \
      "v_mov_b32 %1, " R1 "\n\t"                                                                \
      "v_mov_b32 %2, " R2 "\n\t"                                                                \
      "v_mov_b32 %3, " R3                                                                       \
      : "=&v"(x), "=&v"(y), "=&v"(z), "=&v"(w)                                                  \
      : "s"(m)                                                                                  \
      : "scc");                                                                                 \
    return u32x4{x, y, z, w};                                                                 \
  }
FOGNET_NH_SLOT(0, "v112", "v113", "v114", "v115", "v[112:115]")
FOGNET_NH_SLOT(1, "v116", "v117", "v118", "v119", "v[116:119]")
FOGNET_NH_SLOT(2, "v120", "v121", "v122", "v123", "v[120:123]")
FOGNET_NH_SLOT(3, "v124", "v125", "v126", "v127", "v[124:127]")
FOGNET_NH_SLOT(4, "v152", "v153", "v154", "v155", "v[152:155]")
FOGNET_NH_SLOT(5, "v156", "v157", "v158", "v159", "v[156:159]")
FOGNET_NH_SLOT(6, "v160", "v161", "v162", "v163", "v[160:163]")
FOGNET_NH_SLOT(7, "v164", "v165", "v166", "v167", "v[164:167]")
#undef FOGNET_NH_SLOT
static_assert(kPrefetchOps == 8, "nh_read waits at most for vmcnt(8)");

// S: slot + 4 * register set
template <int S>
__device__ __forceinline__ void nh_prefetch(const RingWord* p) {
  if constexpr (S == 0) nh_prefetch_0(p);
  else if constexpr (S == 1) nh_prefetch_1(p);
  else if constexpr (S == 2) nh_prefetch_2(p);
  else if constexpr (S == 3) nh_prefetch_3(p);
  else if constexpr (S == 4) nh_prefetch_4(p);
  else if constexpr (S == 5) nh_prefetch_5(p);
  else if constexpr (S == 6) nh_prefetch_6(p);
  else nh_prefetch_7(p);
}

// Prefetch stamps are kept per slot, not per node: byte s of the wave-uniform
// `pf` is the tally of the youngest head+1 load issued into slot s's
// registers (by any lane).  A read of slot s waits for that one, which covers
// every older load into the slot: conservative, but needs no per-lane ages
// and no wave reduction.
__device__ __forceinline__ uint32_t set_stamp(uint32_t pf, int s, uint32_t ops) {
  return (pf & ~(0xFFu << (8 * s))) | ((ops & 0xFFu) << (8 * s));
}

// Lanes (of the active ones) with x >= c, as a mask straight from the compare
// (a ballot of a compound bool makes hipcc round-trip it through a VGPR).
__device__ __forceinline__ uint64_t lanes_ge(uint32_t x, uint32_t c) {
  return __builtin_amdgcn_uicmp(x, c, 35 /* ICMP_UGE */);
}

// Wave-level read of slot S's head+1 entry (`need`: wave-uniform, some lane
// uses it) from register set SET (0: v112.., 4: v152..).
template <int S, int SET>
__device__ __forceinline__ u32x4 read_nh(bool need, uint32_t pf, uint32_t ops) {
  const uint32_t m = need ? ((ops - (pf >> (8 * S))) & 0xFFu) : 0xFFu;
  if constexpr (S + SET == 0) return nh_read_0(m);
  else if constexpr (S + SET == 1) return nh_read_1(m);
  else if constexpr (S + SET == 2) return nh_read_2(m);
  else if constexpr (S + SET == 3) return nh_read_3(m);
  else if constexpr (S + SET == 4) return nh_read_4(m);
  else if constexpr (S + SET == 5) return nh_read_5(m);
  else if constexpr (S + SET == 6) return nh_read_6(m);
  else return nh_read_7(m);
}

// Reload the pair holding the head+1 entry of node (slot s, lane): one cache
// line.  Ring stores issued earlier by this wave (any lane) precede it in the
// same in-order memory pipeline, so it observes them.
template <int SET>
__device__ __forceinline__ void refill_nh(int s, const Slot& st, const RingWord* ring, uint32_t qmask, int lane) {
  const RingWord* p = ring + (((n_head(st) + 1u) & qmask) & ~1u);
  const uint64_t only = 1ull << __builtin_amdgcn_readfirstlane(lane);  // lane is wave-uniform
  if constexpr (SET == 0) {
    switch (__builtin_amdgcn_readfirstlane(s)) {
      case 0: nh_refill_0(p, only); break;
      case 1: nh_refill_1(p, only); break;
      case 2: nh_refill_2(p, only); break;
      default: nh_refill_3(p, only); break;
    }
  } else {
    switch (__builtin_amdgcn_readfirstlane(s)) {
      case 0: nh_refill_4(p, only); break;
      case 1: nh_refill_5(p, only); break;
      case 2: nh_refill_6(p, only); break;
      default: nh_refill_7(p, only); break;
    }
  }
}

// ---- issue priority: least replay progress first
//
// The four waves on a SIMD share its VALU, which issues by priority, then age
// (MI355X_MICROARCH.md, "VALU issue is arbitrated ... by priority, then age").
// At equal priority the oldest wave runs nearly unimpeded and the youngest
// gets the leftover slots, so the SIMD's replications finish one after the
// other and the last runs alone, latency-bound (the C3 tail: per-replication
// time min/median/max 14.6/22.5/32.2 M cycles).  Each wave posts its progress
// (fraction of the trace replayed, 2^20 = done) into its hardware slot of a
// board in HBM every kPrioEvery chunks, reads its SIMD's 16 slots and takes
// priority 3 - (number of co-resident waves with less progress), capped at 0:
// the waves advance together and the SIMD stays busy to the end.  Only the
// schedule changes, never a result.
#ifndef FOGNET_PRIO
#define FOGNET_PRIO 2
#endif
#ifndef FOGNET_PRIO_EVERY
#define FOGNET_PRIO_EVERY 32
#endif
constexpr int kPrioEvery = FOGNET_PRIO_EVERY;  // chunks between board updates

__device__ __forceinline__ void set_prio(uint32_t p) {
  switch (p) {
    case 0: __builtin_amdgcn_s_setprio(0); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    default: __builtin_amdgcn_s_setprio(3); break;
  }
}

// This wave's board word: XCC (3 bits) | HW_ID CU/SH/SE (bits 8-15) | SIMD | wave slot.
__device__ __forceinline__ uint32_t board_slot() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return ((xcc & 7u) << 14) | (((hw >> 8) & 0xFFu) << 6) | (((hw >> 4) & 3u) << 4) | (hw & 15u);
}

// Post progress `my` (wave-uniform) and set the priority from the SIMD's slots.
__device__ __forceinline__ void board_update(uint32_t* board, uint32_t slot, uint32_t my, int lane) {
  if (lane == 0) __hip_atomic_store(board + slot, my, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t l = (uint32_t)lane & 15u;
  const uint32_t v = __hip_atomic_load(board + (slot & ~15u) + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t behind = ballot(lane < 16 && l != (slot & 15u) && v < my);  // empty / finished slots hold ~0
  const uint32_t n = (uint32_t)__popcll(behind);
  set_prio(n >= 3u ? 0u : 3u - n);
}

// ---- trace chunk staging (LDS-DMA)
//
// The next 64 publishes {arrive lo, arrive hi, req} are copied global -> LDS
// by three global_load_lds_dword while the current chunk is replayed, so a
// chunk boundary costs an LDS read instead of an HBM round trip.  The copies
// are inline asm (hipcc neither sees nor waits for them): they are tallied in
// `ops` like the head+1 prefetches and waited for by age with wait_vm.  M0 is
// written and restored inside the statement (it is compiler-reserved).  The
// instruction offset is added to the LDS address as well as to the global one
// (LDS = M0 + inst_offset + 4*lane), so the high-dword copy sets
// M0 = base + 0x100 - 4 and lands at base + 0x100 + 4*lane.
#ifdef FOGNET_NT_TRACE
#define FOGNET_TRACE_NT " nt"
#else
#define FOGNET_TRACE_NT ""
#endif
__device__ __forceinline__ void chunk_dma(const int64_t* arrive_c, const int32_t* req_c, uint32_t lane_cl,
                                          uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %5\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %3" FOGNET_TRACE_NT "\n\t"
      "s_add_u32 m0, %5, 0xfc\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %3 offset:4" FOGNET_TRACE_NT "\n\t"
      "s_add_u32 m0, %5, 0x200\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %2, %4" FOGNET_TRACE_NT "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(lane_cl * 8u), "v"(lane_cl * 4u), "s"(arrive_c), "s"(req_c), "s"(lds)
      : "memory");
}
constexpr uint32_t kChunkOps = 3;

// s_waitcnt vmcnt(min(m, 8)) for a wave-uniform m (the immediate needs a branch ladder).
__device__ __forceinline__ void wait_vm(uint32_t m) {
  asm volatile(
      "s_cmp_lt_u32 %0, 8\n\t"
      "s_cbranch_scc1 1f\n\t"
      "s_waitcnt vmcnt(8)\n\t"
      "s_branch 9f\n"
      "1:\n\t"
      "s_cmp_lt_u32 %0, 4\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_cmp_lt_u32 %0, 6\n\t"
      "s_cbranch_scc1 3f\n\t"
      "s_cmp_eq_u32 %0, 6\n\t"
      "s_cbranch_scc1 4f\n\t"
      "s_waitcnt vmcnt(7)\n\t"
      "s_branch 9f\n"
      "4:\n\t"
      "s_waitcnt vmcnt(6)\n\t"
      "s_branch 9f\n"
      "3:\n\t"
      "s_cmp_eq_u32 %0, 4\n\t"
      "s_cbranch_scc1 5f\n\t"
      "s_waitcnt vmcnt(5)\n\t"
      "s_branch 9f\n"
      "5:\n\t"
      "s_waitcnt vmcnt(4)\n\t"
      "s_branch 9f\n"
      "2:\n\t"
      "s_cmp_lt_u32 %0, 2\n\t"
      "s_cbranch_scc1 6f\n\t"
      "s_cmp_eq_u32 %0, 2\n\t"
      "s_cbranch_scc1 7f\n\t"
      "s_waitcnt vmcnt(3)\n\t"
      "s_branch 9f\n"
      "7:\n\t"
      "s_waitcnt vmcnt(2)\n\t"
      "s_branch 9f\n"
      "6:\n\t"
      "s_cmp_eq_u32 %0, 1\n\t"
      "s_cbranch_scc0 8f\n\t"
      "s_waitcnt vmcnt(1)\n\t"
      "s_branch 9f\n"
      "8:\n\t"
      "s_waitcnt vmcnt(0)\n"
      "9:"
      :
      : "s"(m)
      : "scc", "memory");
}

// Cumulative service of the tasks that reached the node before the
// completion (tick `done`, service S) of pending entry head+d0; scans back
// from the newest assignment (tail: cumulative service tl_C, service tl_S;
// entry d's cumulative service is its successor's minus the successor's
// service).  c_self: cumulative service of entry head+d0.
__device__ __forceinline__ uint32_t c_arrived(const Slot& st, const u32x4 nhw, int64_t done, uint32_t S,
                                              uint32_t d0, uint32_t c_self, int64_t dl, uint32_t tl_C,
                                              uint32_t tl_S, const RingWord* ring, uint32_t qmask,
                                              uint32_t& scan) {
  if (arrives_before(st.tl_a, done, dl, S)) return tl_C;
  const uint32_t pend = pending(st);
  uint32_t C = tl_C, S_next = tl_S;  // entry d + 1's
  // entries head+d for d = pend-2 .. d0+1 (the tail, d = pend-1, did not qualify)
  for (uint32_t d = pend - 1u; d-- > d0 + 1u;) {
    RingWord w;
    if (d == 1u) {
      w = nh_word(nhw, nh_odd(st));
    } else {
      PROF(scan += 1u;)
      w = ring[(n_head(st) + d) & qmask];
    }
    C -= S_next;
    if (arrives_before(rw_a(w), done, dl, S)) return C;
    S_next = rw_S(w);
  }
  return c_self;  // only the completing task itself
}

// Apply the advert of the head completion of node k (lane-local): the broker
// view takes busyTime after releaseResource (:232, :254) and the head
// advances; the pair of the new head+1 is prefetched when it starts a new
// pair (an odd new head+1 shares the pair already held).  nhw: the held pair,
// read after its wait.
template <int SL, int SET>
__device__ __forceinline__ void apply_advert(Slot& st, const u32x4 nhw, int k, int64_t dl, int64_t ul, uint32_t tl_C,
                                             uint32_t tl_S, const RingWord* ring, uint32_t qmask, uint32_t ops,
                                             uint32_t& scan) {
  const int64_t hd_done = st.nxt - ul;
  const uint32_t busy =
      c_arrived(st, nhw, hd_done, head_S(st), 0u, st.hd_C, dl, tl_C, tl_S, ring, qmask, scan) - st.hd_C;
  const RingWord w = nh_word(nhw, nh_odd(st));
  st.vkey = (busy << 8) | (uint32_t)k;  // busy < 2^24 (max_s * ring capacity)
  st.cnt += 0x10000u;
  const uint32_t pend = pending(st);
  if (pend == 0u) {
    st.nxt = kNever;
    return;
  }
  const int64_t na = rw_a(w);
  const uint32_t S1 = rw_S(w);
  const int64_t start = na > hd_done ? na : hd_done;
  const int64_t done = start + (int64_t)S1 * kTicksPerSecond;
  st.hd_C += S1;
  st.hd_S = S1;
  st.nxt = done + ul;
  if (pend >= 2u && nh_odd(st) == 0u) {  // the ring holds every pending entry, the tail included
    nh_prefetch<SL + SET>(ring + ((n_head(st) + 1u) & qmask));  // the caller stamps slot SL
  }
}

// Horizons: a lower bound on the tick at which an advert of node j (not the
// current argmin, key best) can change the decision.  No push reaches j
// during the run, so they do not depend on it, and every bound holds for any
// publish tick (a run may continue into the next trace chunk).
//
// Key (b << 8 | j) < best  <=>  b < thr.
__device__ __forceinline__ uint32_t busy_threshold(int j, uint32_t best) {
  return (best >> 8) + ((uint32_t)j < (best & 0xFFu) ? 1u : 0u);
}

// Every pending task of j reached it before its head completes (checked by
// the caller), so completion m advertises busy_m = tl_C - C_m: the value only
// falls by the service completed since the head, and completions are at
// least that many seconds apart.  Needs no ring entry.
__device__ __forceinline__ int64_t horizon_all_in(const Slot& st, int j, uint32_t best, uint32_t tl_C) {
  const uint32_t v1 = tl_C - st.hd_C;
  const uint32_t thr = busy_threshold(j, best);
  if (v1 < thr) return st.nxt;
  const uint32_t need = min(v1 - thr + 1u, 1u << 21);  // cap keeps the sum < 2^63
  return st.nxt + ticks_of(need);
}

// General case: the first two pending completions are evaluated exactly; past
// them the closed form above applies once the queue has fully arrived,
// otherwise the horizon stops at the second.
__device__ __forceinline__ int64_t horizon(const Slot& st, const u32x4 nhw, int j, uint32_t best, uint32_t tl_C,
                                           uint32_t tl_S, int64_t dl, int64_t ul, const RingWord* ring,
                                           uint32_t qmask, uint32_t& scan) {
  const uint32_t pend = pending(st);
  const int64_t hd_done = st.nxt - ul;
  const uint32_t v1 =
      c_arrived(st, nhw, hd_done, head_S(st), 0u, st.hd_C, dl, tl_C, tl_S, ring, qmask, scan) - st.hd_C;
  if (((v1 << 8) | (uint32_t)j) < best) return st.nxt;
  if (pend < 2u) return kNever;
  const RingWord w = nh_word(nhw, nh_odd(st));
  const int64_t na = rw_a(w);
  const uint32_t S1 = rw_S(w), C1 = st.hd_C + S1;
  const int64_t done2 = (na > hd_done ? na : hd_done) + (int64_t)S1 * kTicksPerSecond;
  const int64_t x2 = done2 + ul;
  const uint32_t v2 = c_arrived(st, nhw, done2, S1, 1u, C1, dl, tl_C, tl_S, ring, qmask, scan) - C1;
  if (((v2 << 8) | (uint32_t)j) < best) return x2;
  if (pend == 2u) return kNever;
  if (!arrives_before(st.tl_a, done2, dl, S1)) return x2;
  // fully arrived from completion 2 on: busy_m = v2 - (C_m - C_2), v2 >= thr
  const uint32_t need = min(v2 - busy_threshold(j, best) + 1u, 1u << 21);
  return x2 + ticks_of(need);
}

// Compile-time loop over slots (slot-specific inline asm needs a constant).
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int NPL>
__device__ __forceinline__ uint32_t view_min(const Slot (&st)[NPL]) {
  uint32_t m = st[0].vkey;
#pragma unroll
  for (int s = 1; s < NPL; ++s) m = min(m, st[s].vkey);
  return wave_min_u32(m);
}

// FOGNET_POLICY_EXT_LAT (north-star cost, not in the reference; fognet_hip.h):
// argmin over j of dl_j + (busy_j + min(req / mips_j, 2^20)) * 1e12 in uint64
// ticks (dl_j < 2^50 and busy_j < 2^24 keep it below 2^64), ties -> lowest j.
// The saturation never changes an admissible decision (service <= max_s < 2^16).

template <int NPL>
__device__ __forceinline__ uint32_t ext_argmin(const Slot (&st)[NPL], uint32_t req, const uint32_t* s_dvm,
                                               const uint8_t* s_dvs, const int64_t* s_dl, int N, int lane) {
  uint64_t c[NPL];
  uint64_t m = ~0ull;
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const int j = s * kWave + lane;
    c[s] = ~0ull;
    if (j < N) {
      const uint32_t dvs = s_dvs[j];
      const uint32_t S = min(udiv(req, UDiv{s_dvm[j], (dvs & 1u) | ((dvs >> 1) << 8)}), kExtSatS);
      c[s] = (uint64_t)s_dl[j] + (uint64_t)((st[s].vkey >> 8) + S) * (uint64_t)kTicksPerSecond;
    }
    m = c[s] < m ? c[s] : m;
  }
  m = wave_min_u64(m);
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const uint64_t hit = ballot(s * kWave + lane < N && c[s] == m);
    if (hit) return (uint32_t)(s * kWave + __builtin_ctzll(hit));
  }
  return 0u;
}

// One level of the run's inclusive u32 prefix sum (the element kCtrl names on
// the left; invalid sources read 0).
template <int kCtrl, int kRowMask>
__device__ __forceinline__ uint32_t scan_add_level(uint32_t v) {
  return v + dpp_or_u32<kCtrl, kRowMask>(0u, v);
}

// One level of the run's inclusive i64 prefix maximum.  `tmp` carries the
// DPP destination from level to level: a lane whose source is invalid (or
// whose row is masked off) keeps the value it read at an earlier level, an
// element of an earlier lane that its running maximum already covers (or the
// initial INT64_MIN), so no identity has to be rewritten per level.
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int64_t scan_max_level(int64_t v, int64_t& tmp) {
  tmp = dpp_or_i64<kCtrl, kRowMask>(tmp, v);
  return tmp > v ? tmp : v;
}

// Builder-defined statistics of the north star, after the accumulation (and a
// barrier): histogram counts added into the job histogram, and node energy
// E_j = P_busy_j * B_j + P_idle_j * ((H - B_j 1e12) / 1e12) with IEEE-rounded
// products and sums (no contraction), summed in node order by thread 0.
// Per-node service seconds are integers, so only these final steps round.
__device__ __forceinline__ void stats_finish(const ReplayArgs& A, int r, int64_t H, fognet_rep_stats* S,
                                             const unsigned long long* s_busy, double* s_e, const uint32_t* s_hist,
                                             int tid, int nth) {
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  if (A.hist) {
    for (int h = tid; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += nth)
      if (s_hist[h]) atomicAdd((unsigned long long*)&A.hist[h], (unsigned long long)s_hist[h]);
  }
  if (A.p_busy) {
    for (int j = tid; j < A.N; j += nth) {
      const int64_t B = (int64_t)s_busy[j];
      const double eb = mul_rn(A.p_busy[nbase + j], (double)B);
      const double idle = __ddiv_rn((double)(H - B * kTicksPerSecond), 1e12);
      const double e = add_rn(eb, mul_rn(A.p_idle[nbase + j], idle));
      s_e[j] = e;
      if (A.out_energy) A.out_energy[(size_t)r * (size_t)A.N + j] = e;
    }
    __syncthreads();
    if (tid == 0) {
      double sum = 0.0;
      for (int j = 0; j < A.N; ++j) sum = add_rn(sum, s_e[j]);
      S->energy_j = sum;
    }
  }
}

// ---- statistics epilogue (rep_stats_kernel's pass, fused).  The wave re-reads
// its own replication's outputs (lane l reads tasks l, l + 64, ...; every store
// of the loop precedes it in this wave's memory pipeline: the loop ends with
// vmcnt(0)).  The loop's tail-state LDS is dead now and holds the pass's
// scratch: e_busy aliases s_tld, e_e s_ul, e_hist the chunk stage (>= 128
// words), ab_t [64] i64 + ab_k [64] i32 a dead table of >= 768 B.
template <int NPL>
__device__ __forceinline__ void fused_stats_epilogue(const ReplayArgs& A, int r, int64_t n_done, uint32_t err,
                                                     int64_t* s_tld, const uint32_t* s_tlC, int64_t* s_ul,
                                                     const int64_t* s_dl, uint32_t* e_hist, int64_t* ab_t, int lane) {
  const size_t tbase = (size_t)r * (size_t)A.T;
  unsigned long long* e_busy = reinterpret_cast<unsigned long long*>(s_tld);  // [NPL*64] u64
  double* e_e = reinterpret_cast<double*>(s_ul);                              // [NPL*64] f64
  // A completed replay leaves every node's total service (its tail's
  // cumulative service, exact while n_done * max_s < 2^32) and its last
  // completion (the tail's, FIFO) in the tail state: busy seconds, per-node
  // service for the energy model and `last` then need no per-task work.
  const bool from_tails = err == FOGNET_OK && (uint64_t)n_done * (uint64_t)A.max_s < (1ull << 32);
  Acc acc = acc_identity();
  if (from_tails) {
    for (int j = lane; j < NPL * kWave; j += kWave) {
      const uint32_t B = s_tlC[j];  // 0 for unused nodes and lanes past N
      const int64_t ld = s_tld[j];  // INT64_MIN for unused nodes
      acc.busy += B;
      acc.last = max(acc.last, ld);
      if (A.p_busy) e_busy[j] = B;  // aliases s_tld[j]: read above by this lane
    }
  } else if (A.p_busy) {
    for (int j = lane; j < NPL * kWave; j += kWave) e_busy[j] = 0ull;
  }
  if (A.hist)
    for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave) e_hist[h] = 0u;
  int32_t* const ab_k = reinterpret_cast<int32_t*>(ab_t + kWave);
  ab_t[lane] = INT64_MAX;
  ab_k[lane] = INT32_MAX;
  __syncthreads();
  if (from_tails)
    stats_accumulate<4, false>(A, tbase, (int)n_done, lane, kWave, acc, e_busy, e_hist,
                               [&](int k) { return s_dl[k]; }, ab_t, ab_k);
  else
    stats_accumulate<4>(A, tbase, (int)n_done, lane, kWave, acc, e_busy, e_hist, [&](int k) { return s_dl[k]; },
                        ab_t, ab_k);
  const AbortPt ab = wave_min_abort(AbortPt{ab_t[lane], ab_k[lane]});  // (each lane's own slot)
  acc = wave_merge(acc);
  __syncthreads();
  fognet_rep_stats* S = A.out_stats + r;
  if (lane == 0) write_rep_stats(S, acc, ab, A.ref_abort);
  stats_finish(A, r, n_done > 0 ? acc.last : 0, S, e_busy, e_e, e_hist, lane, kWave);
}

// The replay of replication blockIdx.x (replay_kernel, replay_gen_kernel).
// INL: the statistics are accumulated as the runs are pushed (registers,
// 3 waves/SIMD) instead of by the fused epilogue's re-read of the outputs;
// per-task outputs are still stored unless A.no_task_out.
// GEN (implies INL): generated mode (ReplayArgs::gen_on): the trace chunks
// and node parameters are computed here, and nothing is stored per task.
// r: the replication; slot: its pending-task rings in the workspace.
template <int NPL, int POL, bool GEN, bool INL>
__device__ __forceinline__ void replay_body(const ReplayArgs& A, const int r, const int slot) {
  static_assert(INL || !GEN, "generated mode accumulates in the loop");
  constexpr bool kExt = POL == FOGNET_POLICY_EXT_LAT;
  constexpr int kSet = INL ? 4 : 0;  // prefetch register set
  const int lane = threadIdx.x;
  __shared__ int64_t s_dl[NPL * kWave];
  __shared__ int64_t s_ul[NPL * kWave];
  __shared__ uint32_t s_dvm[NPL * kWave];  // division by the node's MIPS (udiv_magic): multiplier
  __shared__ uint8_t s_dvs[NPL * kWave];   //   and shifts sh1 | sh2 << 1 (sh1 <= 1, sh2 <= 31)
  __shared__ int64_t s_tld[NPL * kWave];   // tail completion tick (INT64_MIN: node never used)
  __shared__ uint32_t s_tlC[NPL * kWave];  // tail cumulative service (mod 2^32)
  __shared__ uint8_t s_tlS[NPL * kWave];   // tail service seconds (< 256 while the replication stays here)
  __shared__ uint32_t s_ch[3 * kWave];     // staged trace chunk: arrive lo | arrive hi | req
  // replay_kernel: the chunk's per-task outputs, one slot per lane (publish c0 + lane), stored to HBM once
  // per chunk (coalesced, one instruction per array) instead of once per run: node (N <= 256), status
  // (0: not pushed), service seconds (start = done - S * 1e12), completion tick
  constexpr bool kBufOut = !GEN && !INL;
  __shared__ uint8_t s_on[kBufOut ? kWave : 1];
  __shared__ uint8_t s_os[kBufOut ? kWave : 1];
  __shared__ uint8_t s_oS[kBufOut ? kWave : 1];
  __shared__ int64_t s_od[kBufOut ? kWave : 1];
  // in-loop statistics (INL): the chunk's pushed tasks, one slot per lane (publish c0 + lane): arrival at
  // the node, completion, service << 8 | status (0: not pushed); accumulated once per chunk
  __shared__ int64_t s_qa[INL ? kWave : 1];
  __shared__ int64_t s_qd[INL ? kWave : 1];
  __shared__ uint32_t s_qs[INL ? kWave : 1];
  // in-loop statistics: the histogram rows (generated mode: in the unused chunk stage)
  __shared__ uint32_t s_hl[(INL && !GEN) ? FOGNET_HIST_METRICS * FOGNET_HIST_BINS : 1];
  // in-loop statistics: the abort point so far (replay_common.h Acc::ab_*), kept in LDS (an overflow is
  // rare; loop-carried registers are not)
  __shared__ int64_t s_ab_tick[1];
  __shared__ int32_t s_ab_task[1];
  // fused epilogue: per-lane abort-point slots (i64 tick + i32 task), in s_dvm when it holds them
  constexpr bool kAbInDvm = NPL * kWave * sizeof(uint32_t) >= kWave * (sizeof(int64_t) + sizeof(int32_t));
  __shared__ int64_t s_abx[(kBufOut && !kAbInDvm) ? kWave * 3 / 2 : 1];
  uint32_t* const s_hs = GEN ? s_ch : s_hl;

  const int T = A.T, N = A.N;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  const uint32_t qmask = (1u << A.q_log2) - 1u;
  GenRep g{};
  if constexpr (GEN) g = gen_rep(A.gen, A.gen_r0 + r, r);
  // (generated: every first advert precedes the first publish by construction)
  const int64_t arrive0 = GEN ? kNever : (T > 0 ? A.arrive[tbase] : kNever);
  const uint32_t lds_ch = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)s_ch;
  uint32_t ch_stamp = 0u;  // `ops` after the staged chunk's copies were issued
  if constexpr (!GEN) {
    if (T > 0) chunk_dma(A.arrive + tbase, A.req + tbase, (uint32_t)min(lane, min(kWave, T) - 1), lds_ch);
  }
  uint64_t ul_max = 0u;  // generated: the largest ul (the first publish follows it)

  // ---- node parameters + preconditions (fognet_hip.h, fognet_batch_in)
  bool bad = false;
  Slot st[NPL];
#pragma unroll
  for (int s = 0; s < NPL; ++s) {
    const int k = s * kWave + lane;
    int64_t d = 0, u = 0;
    int32_t m = 1;
    if (k < N) {
      int64_t ia;
      if constexpr (GEN) {
        gen_node(g, k, m, d, u);
        ia = u;
        ul_max = (uint64_t)u > ul_max ? (uint64_t)u : ul_max;
      } else {
        m = A.mips[nbase + k];
        d = A.dl[nbase + k];
        u = A.ul[nbase + k];
        ia = A.init[nbase + k];
      }
      bad |= (m <= 0) | (d < 0) | (u < 0) | (d > kMaxTick) | (u > kMaxTick) | (ia < u) | (ia >= arrive0);
      if constexpr (kExt) bad |= d >= kExtMaxDl;
    }
    s_dl[k] = d;
    s_ul[k] = u;
    const UDiv dv = udiv_magic((uint32_t)(m > 0 ? m : 1));
    s_dvm[k] = dv.m;
    s_dvs[k] = (uint8_t)((dv.sh & 1u) | ((dv.sh >> 8) << 1));
    // every node's first advert {MIPS, busyTime = 0.0} has reached the broker
    st[s].vkey = k < N ? (uint32_t)k : kNoKey;
    st[s].nxt = kNever;
    st[s].hd_C = 0u;
    st[s].hd_S = 0u;
    st[s].tl_a = 0;
    s_tld[k] = INT64_MIN;
    s_tlC[k] = 0u;
    s_tlS[k] = 0u;
    st[s].cnt = 0u;
  }
  if (INL && A.hist)
    for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave) s_hs[h] = 0u;
  if constexpr (INL) {
    s_qs[lane] = 0u;  // (each lane reads and writes only its own slot)
    if (lane == 0) {
      s_ab_tick[0] = INT64_MAX;
      s_ab_task[0] = INT32_MAX;
    }
  }
  if constexpr (kBufOut) s_os[lane] = 0u;
  __syncthreads();
  int64_t gen_carry = 0;
  if constexpr (GEN) gen_carry = (int64_t)~wave_min_u64(~ul_max) + 1;
  Acc gacc = acc_identity();  // in-loop statistics: this lane's tasks (lane l: tasks l, l + 64, ...)

  uint32_t err = ballot(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;
  if (N <= 0) err = FOGNET_ERR_NO_NODES;

  RingWord* const ring_r = A.ring + (size_t)slot * (size_t)N * ((size_t)qmask + 1u);
  const int q_log2 = A.q_log2;
  // ring of this lane's node in slot s (lanes past N alias node 0: in bounds, never used)
  // Per-lane addresses are rebuilt at each use from wave-uniform bases and an
  // opaque lane index: hoisted out of the loops they would pin 64-bit VGPR
  // pairs for the whole kernel (or spill, and every reload drains vmcnt).
  auto lane_now = [&]() -> uint32_t {
    uint32_t l = (uint32_t)lane;
    asm volatile("" : "+v"(l));
    return l;
  };
  auto ring_s = [&](int s) -> RingWord* {
    const uint32_t k = (uint32_t)(s * kWave) + lane_now();
    return ring_r + ((size_t)(k < (uint32_t)N ? k : 0u) << q_log2);
  };
  uint32_t best = view_min<NPL>(st);
  bool dirty = false;
  int64_t prev_t = INT64_MIN;
  uint32_t max_pend = 0u;
  uint32_t ops = (!GEN && T > 0) ? kChunkOps : 0u;  // tally of issued vector-memory instructions (see kPrefetchOps)
  uint32_t pf = 0u;                       // per-slot stamps of the youngest head+1 loads (set_stamp)
  ch_stamp = ops;
  int64_t n_done = 0;
  uint32_t scan = 0u;  // profile builds: ring entries read by c_arrived (per lane)
#if FOGNET_REPLAY_PROFILE == 3
  // timeline probe (tools/c3_timeline.py): the wave's start, replay end and epilogue end (s_memtime)
  const uint64_t tl_t0 = __builtin_amdgcn_s_memtime();
#endif
#if FOGNET_REPLAY_PROFILE == 2
  uint64_t p_t[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t p_start = __builtin_amdgcn_s_memtime();
  uint64_t p_last = p_start;
#endif
#if FOGNET_REPLAY_PROFILE == 1
  uint64_t p_iter = 0, p_advit = 0, p_adv = 0, p_end_k = 0, p_end_j = 0, p_end_c = 0, p_hz = 0, p_refill = 0, p_w0 = 0, p_rd = 0,
           p_chunks = 0, p_pk0 = 0, p_resume = 0, p_same = 0, p_endh_same = 0;
  int prev_k = -1;
  bool prev_end_h = false;
  auto young = [&](int s, bool need) { return ballot(need) && ((ops - (pf >> (8 * s))) & 0xFFu) < 2u; };
#endif
  // A run that consumed the rest of its chunk continues into the next one
  // while the publishes stay within its horizon E_carry (argmin unchanged).
  bool carry = false;
  int64_t E_carry = 0;
  // issue priority (replay_kernel only; see board_update)
  constexpr bool kPrio = FOGNET_PRIO != 0 && !GEN && !INL;
  uint32_t b_slot = 0u;
  float b_scale = 0.0f;
  if constexpr (kPrio) {
    b_slot = board_slot();
    b_scale = 1048576.0f / (float)(T > 0 ? T : 1);
  }

  for (int c0 = 0; c0 < T && err == FOGNET_OK; c0 += kWave) {
    const int cnt = min(kWave, T - c0);
    const bool live = lane < cnt;
    int64_t ca;
    int32_t cr;
    if constexpr (GEN) {
      gen_chunk(g, c0, T, lane, gen_carry, ca, cr);
    } else {
      wait_vm((ops - ch_stamp) & 0xFFu);  // the staged chunk has landed in LDS
      const uint32_t l_ch = lane_now();
      ca = live ? (int64_t)(((uint64_t)s_ch[kWave + l_ch] << 32) | s_ch[l_ch]) : kNever;
      cr = live ? (int32_t)s_ch[2 * kWave + l_ch] : 0;
    }
    PROF(p_chunks++;)
    if constexpr (kPrio) {
      if (((c0 >> 6) & (kPrioEvery - 1)) == 0) {
        const uint32_t my = __builtin_amdgcn_readfirstlane((uint32_t)((float)c0 * b_scale));
#if FOGNET_PRIO == 2
        if (A.board) board_update(A.board, b_slot, my, lane);
#else
        set_prio(3u - min(my >> 18, 3u));  // quartile of the trace
#endif
      }
    }
    TMARK(0)
    // trace preconditions: nondecreasing ticks, requirement >= 0, ticks < 2^61
    const int64_t prv = dpp_or_i64<kDppWaveShr1>(prev_t, ca);  // lane 0 gets prev_t
    if (ballot(live && (ca < prv || cr < 0 || ca > kMaxTick))) {
      err = FOGNET_ERR_ARG;
      break;
    }
    prev_t = readlane_i64(ca, cnt - 1);
    const int64_t t_last = prev_t;  // only picks which horizons are evaluated exactly
    if (!GEN && c0 + kWave < T) {  // stage the next chunk (ca/cr were consumed above: LDS reads are done)
      const int cn = min(kWave, T - c0 - kWave);
      chunk_dma(A.arrive + tbase + c0 + kWave, A.req + tbase + c0 + kWave, (uint32_t)min(lane, cn - 1), lds_ch);
      ops += kChunkOps;
      ch_stamp = ops;
    }
    TMARK(0)

    int jp = 0;
    while (jp < cnt) {
      const int64_t t_p = readlane_i64(ca, jp);
      PROF(p_iter++;)
      const bool resume = !kExt && carry && t_p <= E_carry;
      carry = false;
      int64_t E = E_carry;
      if (!resume) {
        // 1) completion adverts that reached the broker strictly before t_p.
        //    Adverts of different nodes commute (each sets only its node's
        //    key), so rounds go over the slots round-robin: a node's next
        //    head+1 wait is then covered by the other slots' work.
        for (;;) {
          bool any = false;
          static_for<0, NPL>([&](auto sc) {
            constexpr int s = decltype(sc)::value;
            const bool due = st[s].nxt < t_p;
            const uint64_t dm = ballot(due);
            if (!dm) return;
            const uint32_t pd = pending(st[s]);
            any = true;
            dirty = true;
            PROF(p_advit++; p_adv += __popcll(ballot(due)); p_rd++; p_w0 += young(s, due && pending(st[s]) >= 2u);)
            TMARK(1)
            const u32x4 nhw = read_nh<s, kSet>((dm & lanes_ge(pd, 2u)) != 0, pf, ops);
            TMARK(8)
            // apply_advert prefetches the pair of head+2 where >= 3 are pending
            // and head+2 starts a pair (head even): tally it first, so the stamp
            // already counts the load itself
            if (dm & lanes_ge(pd, 3u) & ballot((st[s].cnt & 0x10000u) == 0u)) {
              ops += 1u;
              pf = set_stamp(pf, s, ops);
            }
            if (due) {
              const int k = s * kWave + lane;
              apply_advert<s, kSet>(st[s], nhw, k, s_dl[k], s_ul[k], s_tlC[k], s_tlS[k], ring_s(s), qmask, ops,
                                    scan);
            }
          });
          if (!any) break;
        }
        TMARK(1)
        if constexpr (kExt) {
          // 2') per-publish argmin of the extension cost; every run is one publish
          best = ext_argmin<NPL>(st, readlane_u32((uint32_t)cr, jp), s_dvm, s_dvs, s_dl, N, lane);
        } else {
        // 2) argmin over the advertised view (ties -> lowest index)
        if (dirty) {
          best = view_min<NPL>(st);
          dirty = false;
        }
        TMARK(2)
        const int k = (int)(best & 0xFFu);
        PROF(p_same += k == prev_k; p_endh_same += prev_end_h && k == prev_k;)

        // 3) run horizon: earliest advert that could change the decision.
        //    Only nodes whose key can drop below best (busy >= 0) matter.
        int64_t e_lane = kNever;
        static_for<0, NPL>([&](auto sc) {
          constexpr int s = decltype(sc)::value;
          const int j = s * kWave + lane;
          const uint32_t pd = pending(st[s]);
          const bool rel = j < N && j != k && (uint32_t)j < best && pd >= 1u;
          bool deep = false;
          if (rel) {
            const uint32_t tlC_j = s_tlC[j];
            if (arrives_before(st[s].tl_a, st[s].nxt - s_ul[j], s_dl[j], head_S(st[s]))) {
              const int64_t h = horizon_all_in(st[s], j, best, tlC_j);
              e_lane = h < e_lane ? h : e_lane;
            } else if (st[s].nxt < t_last) {
              deep = true;
            } else {
              e_lane = st[s].nxt < e_lane ? st[s].nxt : e_lane;  // beyond this chunk: its first advert
            }
          }
          const uint64_t dm = ballot(deep);
          if (dm) {
            PROF(p_hz++; p_rd++; p_w0 += young(s, deep && pending(st[s]) >= 2u);)
            TMARK(3)
            const u32x4 nhw = read_nh<s, kSet>((dm & lanes_ge(pd, 2u)) != 0, pf, ops);
            TMARK(9)
            if (deep) {
              const int64_t h =
                  horizon(st[s], nhw, j, best, s_tlC[j], s_tlS[j], s_dl[j], s_ul[j], ring_s(s), qmask, scan);
              e_lane = h < e_lane ? h : e_lane;
            }
          }
        });
        E = (int64_t)wave_min_u64((uint64_t)e_lane);  // all candidates are >= 0
        }  // REF_V3
      } else {
        PROF(p_resume++;)
      }
      const int k = (int)(best & 0xFFu);
      const int ks = k / kWave, kl = k % kWave;
      PROF(const int64_t E_other = E;)
      TMARK(3)

      // node k: parameters and tail state (uniform)
      const int64_t dl_k = s_dl[k], ul_k = s_ul[k];
      const uint32_t dvs_k = s_dvs[k];
      const UDiv div_k{s_dvm[k], (dvs_k & 1u) | ((dvs_k >> 1) << 8)};
      const uint32_t tlC_k = s_tlC[k], tlS_k = s_tlS[k];
      const int64_t tld_k = s_tld[k];
      uint32_t cnt_k = 0u;
      int64_t nxt_k = 0;
#pragma unroll
      for (int s = 0; s < NPL; ++s) {
        if (s == ks) {
          cnt_k = readlane_u32(st[s].cnt, kl);
          nxt_k = readlane_i64(st[s].nxt, kl);
        }
      }
      const uint32_t pend_k = ((cnt_k & 0xFFFFu) - (cnt_k >> 16)) & 0xFFFFu;
      if (resume) {
        // E_carry already holds k's own bound
      } else if (pend_k > 0u) {
        E = nxt_k < E ? nxt_k : E;  // k's own next advert changes its key
      } else {
        // the run's first task becomes k's head: its advert ends the run
        const uint32_t s_p = udiv(readlane_u32((uint32_t)cr, jp), div_k);
        const int64_t a_p = t_p + dl_k;
        const int64_t done_p = (a_p > tld_k ? a_p : tld_k) + (int64_t)(s_p & 0xFFFFu) * kTicksPerSecond;
        const int64_t x_p = done_p + ul_k;
        E = x_p < E ? x_p : E;
      }

      // 4) the run: publishes jp .. jq-1 with tick <= E all go to node k
      const bool in_run = kExt ? lane == jp : ((lane >= jp && lane < cnt && ca <= E) || lane == jp);
      const uint64_t run_mask = ballot(in_run);
      const int L = __popcll(run_mask);
      const int jq = jp + L;

      // 5) FIFO recurrence over the run: done_m = max(a_m, done_{m-1}) + S_m.
      //    Non-run lanes carry the identities (S = 0, X = INT64_MIN); DPP row
      //    shifts and row broadcasts fill invalid sources with them.
      uint32_t S = 0u;
      int64_t a = 0, dd = 0;
      bool lerr = false, lwide = false;
      if (in_run) {
        S = udiv((uint32_t)cr, div_k);  // double tskTime = requiredMIPS / MIPS (:276)
        a = ca + dl_k;
        dd = (int64_t)S * kTicksPerSecond;
        lerr = a > kMaxTick;
        // beyond this kernel's 24-bit busy key or its 8-B ring entry: the wide kernel replays it
        lwide = S > A.max_s || S > kRingSMask || a > kRingAMax;
      }
      //    Unrolled: with P_m = sum_{i<=m} S_i 1e12 (a prefix sum) and
      //    X_m = a_m - P_{m-1},  done_m = max(done_before_run, max_{i<=m} X_i) + P_m,
      //    i.e. one u32 prefix sum and one i64 prefix max over the wave.
      //    Unsigned arithmetic: rejected lanes (lerr) may wrap, never UB.
      uint32_t Cs = S;
      Cs = scan_add_level<0x111, 0xF>(Cs);  // row_shr:1
      Cs = scan_add_level<0x112, 0xF>(Cs);  // row_shr:2
      Cs = scan_add_level<0x114, 0xF>(Cs);  // row_shr:4
      Cs = scan_add_level<0x118, 0xF>(Cs);  // row_shr:8
      Cs = scan_add_level<0x142, 0xA>(Cs);  // row_bcast:15
      Cs = scan_add_level<0x143, 0xC>(Cs);  // row_bcast:31
      const int64_t base_done = tld_k;  // INT64_MIN when k never ran a task
      int64_t done;
      uint32_t status;
      // Queued run (the common case under the stale view's herding): k is busy
      // past the run's last arrival, so every task queues behind it and
      // done_m = base_done + P_m; no prefix maximum, no status tests.
      if (base_done > (int64_t)((uint64_t)readlane_i64(ca, jq - 1) + (uint64_t)dl_k)) {
        done = (int64_t)((uint64_t)base_done + (uint64_t)ticks_of(Cs));
        status = 4u;  // busy: "task queued" (:304-313)
      } else {
        int64_t X = in_run ? (int64_t)((uint64_t)a - (uint64_t)ticks_of(Cs - S)) : INT64_MIN;
        int64_t xt = INT64_MIN;
        X = scan_max_level<0x111, 0xF>(X, xt);
        X = scan_max_level<0x112, 0xF>(X, xt);
        X = scan_max_level<0x114, 0xF>(X, xt);
        X = scan_max_level<0x118, 0xF>(X, xt);
        X = scan_max_level<0x142, 0xA>(X, xt);
        X = scan_max_level<0x143, 0xC>(X, xt);
        const int64_t dmax = base_done > X ? base_done : X;
        done = (int64_t)((uint64_t)dmax + (uint64_t)ticks_of(Cs));
        // previous task on node k: the run's previous lane, or k's tail
        const int64_t done_up = dpp_or_i64<kDppWaveShr1>(0, done);
        const uint32_t S_up = dpp_or_u32<kDppWaveShr1>(0u, S);
        const int64_t prev_done = lane == jp ? base_done : done_up;
        const uint32_t prev_S = lane == jp ? tlS_k : S_up;
        if (prev_done < a) {
          status = 5u;  // idle: "task assigned" (:282-301)
        } else if (prev_done > a) {
          status = 4u;  // busy: "task queued" (:304-313)
        } else {        // completion of the previous task at the same tick
          status = (dl_k < (int64_t)prev_S * kTicksPerSecond) ? 5u : 4u;
        }
      }
      const int64_t start = done - dd;
      lerr = lerr || (in_run && done > kMaxTick);
      if (ballot(lerr)) {
        err = FOGNET_ERR_ARG;
        break;
      }
      // a node with more than ring-capacity pending tasks, or a service time
      // the 24-bit busy key cannot hold: hand the replication to the wide
      // kernel (unbounded per-node chains), which replays it from the start
      if (ballot(lwide) || pend_k + (uint32_t)L - 1u > qmask) {
        err = kNeedsWide;
        break;
      }
      TMARK(4)
      // ring entries (consecutive slots of node k's ring) and per-task outputs
      RingWord* const ring_k = ring_r + ((size_t)k << q_log2);
      if (in_run) {
        ring_k[((cnt_k & 0xFFFFu) + (uint32_t)(lane - jp)) & qmask] = ((uint64_t)a << kRingSBits) | S;
        if constexpr (INL) {
          // the task's statistics: accumulated at the end of the chunk, with every pushed lane at
          // once (a run pushes 1..64 lanes; S < 256 in a replay that stays in this kernel)
          s_qa[lane] = a;
          s_qd[lane] = done;
          s_qs[lane] = (S << 8) | status;
        }
        if constexpr (kBufOut) {
          s_on[lane] = (uint8_t)k;
          s_os[lane] = (uint8_t)status;
          s_oS[lane] = (uint8_t)S;
          s_od[lane] = done;
        } else if (!GEN && !(INL && A.no_task_out)) {
          // chunk bases are wave-uniform (SGPR) and the lane index a 32-bit
          // offset, so no per-lane 64-bit addresses stay live across the chunk
          const size_t o = tbase + (size_t)c0;
          const uint32_t l = lane_now();
          // nontemporal: the outputs are re-read only by the epilogue, long
          // after they left L2; the ring's head lines keep the cache (-4 %)
          __builtin_nontemporal_store(k, (A.out_node + o) + l);
          __builtin_nontemporal_store((uint8_t)status, (A.out_status + o) + l);
          __builtin_nontemporal_store(start, (A.out_start + o) + l);
          __builtin_nontemporal_store(done, (A.out_done + o) + l);
        }
      }
      // the ring store (+ the four output stores)
      ops += (kBufOut || GEN || (INL && A.no_task_out)) ? 1u : 5u;
      TMARK(5)

      // 6) node k's state after the run
      const int lz = jq - 1;
      const int64_t a_z = readlane_i64(a, lz), done_z = readlane_i64(done, lz);
      const uint32_t C_z = readlane_u32(tlC_k + Cs, lz), S_z = readlane_u32(S, lz);
      const int64_t done_f = readlane_i64(done, jp);
      const uint32_t C_f = readlane_u32(tlC_k + Cs, jp), S_f = readlane_u32(S, jp);
#pragma unroll
      for (int s = 0; s < NPL; ++s) {
        if (s == ks) {
          if (lane == kl) {
            if (pend_k == 0u) {
              st[s].hd_C = C_f;
              st[s].hd_S = S_f;
              st[s].nxt = done_f + ul_k;
            }
            st[s].tl_a = a_z;
            s_tld[k] = done_z;
            s_tlC[k] = C_z;
            s_tlS[k] = S_z;
            st[s].cnt = (cnt_k & 0xFFFF0000u) | ((cnt_k + (uint32_t)L) & 0xFFFFu);
          }
          // the run wrote into the held pair (entry head+1, or head+2 when it
          // shares head+1's pair): reload it (uniform control flow, one lane)
          const uint32_t pl = pend_k + (uint32_t)L;
          if ((pend_k <= 1u && pl >= 2u) || ((cnt_k & 0x10000u) != 0u && pend_k <= 2u && pl >= 3u)) {
            refill_nh<kSet>(s, st[s], ring_s(s), qmask, kl);
            PROF(p_refill++;)
            ops += 1u;
            pf = set_stamp(pf, s, ops);  // the stamp counts the refill itself
          }
        }
      }
      const uint32_t pend_after = pend_k + (uint32_t)L;
      max_pend = pend_after > max_pend ? pend_after : max_pend;
      n_done += L;
      if (!kExt && jq == cnt) {  // the chunk is used up and E still bounds the decision
        carry = true;
        E_carry = E;
      }
      TMARK(6)
      PROF(p_pk0 += pend_k == 0u; if (jq >= cnt) p_end_c++; else if (E == E_other) p_end_j++; else p_end_k++;
           prev_k = k; prev_end_h = jq < cnt && E == E_other;)
      jp = jq;
    }
    if constexpr (kBufOut) {
      // the chunk's outputs (also after an error ended it: the tasks pushed so far)
      const uint32_t so = s_os[lane];
      if (ballot(so != 0u)) {
        if (so != 0u) {
          const size_t o = tbase + (size_t)c0;
          const uint32_t l = lane_now();
          const int64_t dn = s_od[lane];
          // nontemporal: the outputs are re-read only by the epilogue, long
          // after they left L2; the ring's head lines keep the cache
          __builtin_nontemporal_store((int32_t)s_on[lane], (A.out_node + o) + l);
          __builtin_nontemporal_store((uint8_t)so, (A.out_status + o) + l);
          __builtin_nontemporal_store(dn - ticks_of(s_oS[lane]), (A.out_start + o) + l);
          __builtin_nontemporal_store(dn, (A.out_done + o) + l);
          s_os[lane] = 0u;
        }
        ops += 4u;
      }
    }
    if constexpr (INL) {
      // the chunk's statistics (the fused epilogue's, rep_stats_kernel's), also after an
      // error ended it (the tasks pushed so far)
      const uint32_t qs = s_qs[lane];
      bool ovf = false;  // this lane's queueTime emission overflows: the reference's abort point
      int64_t st_o = 0;
      if (qs != 0u) {
        const int64_t a_q = s_qa[lane], done_q = s_qd[lane];
        const int64_t resp = done_q - ca;
        add_moment(gacc.rs_lo, gacc.rs_hi, gacc.rq_lo, gacc.rq_hi, (uint64_t)resp);
        gacc.rmin = min(gacc.rmin, resp);
        gacc.rmax = max(gacc.rmax, resp);
        if (A.hist) atomicAdd(&s_hs[FOGNET_HIST_BINS + hist_bin(resp)], 1u);
        if ((qs & 0xFFu) == 4u) {
          gacc.n4 += 1u;
          st_o = done_q - ticks_of(qs >> 8);
          ovf = !acc_qtime(gacc.qs_lo, gacc.qs_hi, gacc.qq_lo, gacc.qq_hi, gacc.qq_top, gacc.qmin, gacc.qmax,
                           gacc.nqt, gacc.nqo, st_o, a_q, A.hist ? s_hs : nullptr);
        } else {
          gacc.n5 += 1u;
        }
        s_qs[lane] = 0u;
      }
      if (ballot(ovf)) {  // rare: the chunk's earliest overflowing emission (ticks >= 0), then the lowest index
        const AbortPt m = wave_min_abort(ovf ? AbortPt{st_o, c0 + lane} : abort_none());
        if (lane == 0) abort_min(s_ab_tick[0], s_ab_task[0], m.tick, m.task);
      }
    }
    TMARK(7)  // (profile builds: the chunk's output flush and statistics)
  }
  // drain the inline-asm prefetches before the wave retires
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (kPrio && FOGNET_PRIO == 2) {  // this slot is free again
    if (A.board && lane == 0) __hip_atomic_store(A.board + b_slot, ~0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }

#if FOGNET_REPLAY_PROFILE == 2
  TMARK(7)
#endif
#if FOGNET_REPLAY_PROFILE == 1
  uint64_t p_scan = 0;
  for (int l = 0; l < kWave; ++l) p_scan += readlane_u32(scan, l);
#endif
  if (lane == 0 && err == kNeedsWide && A.wide_list) A.wide_list[atomicAdd(A.wide_count, 1)] = r;
  if (lane == 0 && A.out_stats) {
    fognet_rep_stats* S = A.out_stats + r;
    S->n_tasks = n_done;
    S->max_pending = (int32_t)max_pend;
    S->status = (int32_t)err;
    S->events = 2 * (int64_t)N + 4 * n_done;
#if FOGNET_REPLAY_PROFILE == 2
    S->n_queued = p_t[0];
    S->n_started = p_t[1];
    S->last_tick = p_t[2];
    S->queue_min_raw = p_t[3];
    S->queue_max_raw = p_t[4];
    S->resp_min_ticks = p_t[5];
    S->resp_max_ticks = p_t[6];
    S->queue_sum_lo = p_t[7];
    S->queue_sq_lo = p_t[8];
    S->queue_sq_hi = p_t[9];
    S->queue_sum_hi = p_last - p_start;
#endif
#if FOGNET_REPLAY_PROFILE == 1
    S->n_queued = p_iter;
    S->n_started = p_advit;
    S->last_tick = p_adv;
    S->queue_min_raw = p_scan;
    S->queue_max_raw = p_end_k;
    S->resp_min_ticks = p_hz;
    S->resp_max_ticks = p_refill;
    S->queue_sum_lo = p_w0;
    S->queue_sum_hi = p_rd;
    S->queue_sq_lo = p_chunks;
    S->queue_sq_hi = p_end_j;
    S->resp_sum_hi = p_end_c;
    S->resp_sq_lo = p_resume;
    S->resp_sum_lo = p_pk0;
    S->busy_s = (int64_t)p_same;
    S->resp_sq_hi = p_endh_same;
#endif
  }
#if FOGNET_REPLAY_PROFILE == 3
  const uint64_t tl_t1 = __builtin_amdgcn_s_memtime();
#endif
#if !defined(FOGNET_REPLAY_PROFILE) || FOGNET_REPLAY_PROFILE == 0 || FOGNET_REPLAY_PROFILE == 3
  if constexpr (INL) {
    if (A.out_stats && err != kNeedsWide) {
      // busy seconds, per-node service (energy) and `last` from the node
      // tails (exact: the host takes this path only while T * max service < 2^32), the rest from
      // the loop's accumulators
      unsigned long long* e_busy = reinterpret_cast<unsigned long long*>(s_tld);  // [NPL*64] u64
      double* e_e = reinterpret_cast<double*>(s_ul);                              // [NPL*64] f64
      for (int j = lane; j < NPL * kWave; j += kWave) {
        const uint32_t B = s_tlC[j];
        const int64_t ld = s_tld[j];
        gacc.busy += B;
        gacc.last = max(gacc.last, ld);
        if (A.p_busy) e_busy[j] = B;  // aliases s_tld[j]: read above by this lane
      }
      gacc = wave_merge(gacc);
      __syncthreads();
      fognet_rep_stats* S = A.out_stats + r;
      if (lane == 0) write_rep_stats(S, gacc, AbortPt{s_ab_tick[0], s_ab_task[0]}, A.ref_abort);
      stats_finish(A, r, n_done > 0 ? gacc.last : 0, S, e_busy, e_e, s_hs, lane, kWave);
    }
  } else if (A.fuse_stats && A.out_stats && err != kNeedsWide) {
    fused_stats_epilogue<NPL>(A, r, n_done, err, s_tld, s_tlC, s_ul, s_dl, s_ch,
                              reinterpret_cast<int64_t*>(kAbInDvm ? (void*)s_dvm : (void*)s_abx), lane);
  }
#endif
#if FOGNET_REPLAY_PROFILE == 3
  if constexpr (!GEN && !INL) {
    const uint64_t tl_t2 = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (lane == 0 && T >= 4) {  // (over the replication's first outputs: a timing probe only)
      A.out_done[tbase + 0] = (int64_t)tl_t0;
      A.out_done[tbase + 1] = (int64_t)tl_t1;
      A.out_done[tbase + 2] = (int64_t)tl_t2;
      A.out_done[tbase + 3] = (int64_t)board_slot();
    }
  }
#endif
}

// 4 waves per SIMD (<= 128 VGPRs) and <= 10 KiB of LDS (160 KiB / 16): 16
// replications resident per CU, so the 4096-replication sweep runs in a single
// wave of workgroups on 256 CUs.  (11 KiB of LDS admits only 14 per CU, and
// the last 512 replications then run as a second, mostly idle round.)
template <int NPL, int POL>
__global__ __launch_bounds__(64, 4) __attribute__((amdgpu_num_vgpr(kNhBase / 2))) void replay_kernel(ReplayArgs A) {
  replay_body<NPL, POL, false, false>(A, blockIdx.x, blockIdx.x);
}

// Statistics in the loop (ReplayArgs::inloop): 3 waves per SIMD like the
// generated mode, the trace and outputs as replay_kernel's.
template <int NPL, int POL>
__global__ __launch_bounds__(64, 3) __attribute__((amdgpu_num_vgpr(kNhBaseGen / 2))) void replay_inl_kernel(
    ReplayArgs A) {
  replay_body<NPL, POL, false, true>(A, blockIdx.x, blockIdx.x);
}

// Generated mode: 3 waves per SIMD (168 VGPRs: the statistics accumulators stay
// in registers through the loop), prefetch registers v152..v167.  A grid of
// at most the resident workgroups takes the replications from a work
// counter (A.queue, zeroed before the launch), so the rings are per workgroup
// and a million-replication job is one launch without a tail per block; every
// workgroup leaves once the counter has passed R.
template <int NPL, int POL>
__global__ __launch_bounds__(64, 3) __attribute__((amdgpu_num_vgpr(kNhBaseGen / 2))) void replay_gen_kernel(
    ReplayArgs A) {
  for (;;) {
    int next = 0;
    if (threadIdx.x == 0) next = atomicAdd(A.queue, 1);
    const int r = __builtin_amdgcn_readlane(next, 0);
    if (r >= A.R) break;
    replay_body<NPL, POL, true, true>(A, r, blockIdx.x);
    __syncthreads();  // LDS reuse by the next replication
  }
}

constexpr int kStatThreads = 256;

// Standalone statistics pass over the replay outputs (fognet_rep_stats_dev);
// fognet_run_batch_dev fuses the same pass into replay_kernel instead.
__global__ __launch_bounds__(kStatThreads) void rep_stats_kernel(ReplayArgs A) {
  const int r = blockIdx.x;
  __shared__ Acc s_acc[kStatThreads];
  __shared__ int64_t s_abt[kStatThreads];  // per thread: the abort point (AbortPt), rare updates
  __shared__ int32_t s_abk[kStatThreads];
  __shared__ unsigned long long s_busy[kWave * kMaxNodesPerLane];  // service seconds per node
  __shared__ double s_e[kWave * kMaxNodesPerLane];
  __shared__ uint32_t s_hist[FOGNET_HIST_METRICS * FOGNET_HIST_BINS];
  fognet_rep_stats* S = A.out_stats + r;
  const int32_t n = (int32_t)S->n_tasks;  // written by replay_kernel
  const size_t tbase = (size_t)r * (size_t)A.T;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  for (int j = threadIdx.x; j < kWave * kMaxNodesPerLane; j += kStatThreads) s_busy[j] = 0ull;
  for (int h = threadIdx.x; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kStatThreads) s_hist[h] = 0u;
  s_abt[threadIdx.x] = INT64_MAX;
  s_abk[threadIdx.x] = INT32_MAX;
  __syncthreads();
  Acc a = acc_identity();
  stats_accumulate<2>(A, tbase, n, threadIdx.x, kStatThreads, a, s_busy, s_hist,
                      [&](int k) { return A.dl[nbase + k]; }, s_abt, s_abk);
  s_acc[threadIdx.x] = a;
  __syncthreads();
  for (int w = kStatThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) {
      acc_merge(s_acc[threadIdx.x], s_acc[threadIdx.x + w]);
      abort_min(s_abt[threadIdx.x], s_abk[threadIdx.x], s_abt[threadIdx.x + w], s_abk[threadIdx.x + w]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) write_rep_stats(S, s_acc[0], AbortPt{s_abt[0], s_abk[0]}, A.ref_abort);
  stats_finish(A, r, n > 0 ? s_acc[0].last : 0, S, s_busy, s_e, s_hist, threadIdx.x, kStatThreads);
}

}  // namespace

template <int POL>
void launch_replay_pol(const ReplayArgs& a, hipStream_t s) {
  const int npl = (a.N + kWave - 1) / kWave;
  if (a.gen_on) {
    const dim3 grid(a.R < a.gen_slots ? a.R : a.gen_slots);
    if (npl <= 1)
      hipLaunchKernelGGL((replay_gen_kernel<1, POL>), grid, dim3(kWave), 0, s, a);
    else if (npl == 2)
      hipLaunchKernelGGL((replay_gen_kernel<2, POL>), grid, dim3(kWave), 0, s, a);
    else
      hipLaunchKernelGGL((replay_gen_kernel<4, POL>), grid, dim3(kWave), 0, s, a);
    return;
  }
  if (a.inloop) {
    if (npl <= 1)
      hipLaunchKernelGGL((replay_inl_kernel<1, POL>), dim3(a.R), dim3(kWave), 0, s, a);
    else if (npl == 2)
      hipLaunchKernelGGL((replay_inl_kernel<2, POL>), dim3(a.R), dim3(kWave), 0, s, a);
    else
      hipLaunchKernelGGL((replay_inl_kernel<4, POL>), dim3(a.R), dim3(kWave), 0, s, a);
    return;
  }
  if (npl <= 1) {
    hipLaunchKernelGGL((replay_kernel<1, POL>), dim3(a.R), dim3(kWave), 0, s, a);
  } else if (npl == 2) {
    hipLaunchKernelGGL((replay_kernel<2, POL>), dim3(a.R), dim3(kWave), 0, s, a);
  } else {
    hipLaunchKernelGGL((replay_kernel<4, POL>), dim3(a.R), dim3(kWave), 0, s, a);
  }
}

hipError_t launch_replay(const ReplayArgs& a, hipStream_t s) {
  if (a.policy == FOGNET_POLICY_EXT_LAT)
    launch_replay_pol<FOGNET_POLICY_EXT_LAT>(a, s);
  else
    launch_replay_pol<FOGNET_POLICY_REF_V3>(a, s);
  return hipGetLastError();
}

hipError_t launch_rep_stats(const ReplayArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(rep_stats_kernel, dim3(a.R), dim3(kStatThreads), 0, s, a);
  return hipGetLastError();
}

}  // namespace fognet
