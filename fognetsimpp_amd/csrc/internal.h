// internal.h — device helpers and kernel entry points shared by the
// libfognet_hip translation units.  gfx950 (CDNA4, wave64) only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fognet_hip.h"

namespace fognet {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int64_t kTicksPerSecond = FOGNET_TICKS_PER_SECOND;
constexpr int kMaxNodesPerLane = 4;  // N <= 256 in the register-resident replay kernel

// ---------------------------------------------------------------- lane moves

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}

__device__ __forceinline__ int64_t readlane_i64(int64_t v, int lane) {
  const uint32_t lo = readlane_u32((uint32_t)(uint64_t)v, lane);
  const uint32_t hi = readlane_u32((uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// DPP move of a 32-bit value (bound_ctrl: out-of-row sources read 0; every
// pattern used below stays inside a row of 16 lanes).
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kCtrl, 0xF, 0xF, true);
}

template <int kCtrl>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const uint32_t lo = dpp_u32<kCtrl>((uint32_t)v);
  const uint32_t hi = dpp_u32<kCtrl>((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// DPP move that leaves `old` where the source lane is invalid or the row is
// masked off (bound_ctrl off): shifts with a fill value and the row
// broadcasts of a wave scan.
//   row_shr:n 0x110+n (within rows of 16)   wave_shr:1 0x138 (whole wave)
//   row_bcast:15 0x142 (lane 15 of each row -> next row; rows 1,3: mask 0xA)
//   row_bcast:31 0x143 (lane 31 -> rows 2,3: mask 0xC)
template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ uint32_t dpp_or_u32(uint32_t old, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, kCtrl, kRowMask, 0xF, false);
}

template <int kCtrl, int kRowMask = 0xF>
__device__ __forceinline__ int64_t dpp_or_i64(int64_t old, int64_t v) {
  const uint32_t lo = dpp_or_u32<kCtrl, kRowMask>((uint32_t)(uint64_t)old, (uint32_t)(uint64_t)v);
  const uint32_t hi = dpp_or_u32<kCtrl, kRowMask>((uint32_t)((uint64_t)old >> 32), (uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

constexpr int kDppWaveShr1 = 0x138;

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return b < a ? b : a; }

// Minimum of a u64 over the 64 lanes; result is wave-uniform.  Must be called
// with every lane active.  Four in-row DPP butterflies (quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror, row_mirror) leave each row of 16 holding its
// minimum; the four row minima are then combined on the scalar side.
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
  v = umin64(v, dpp_u64<0xB1>(v));
  v = umin64(v, dpp_u64<0x4E>(v));
  v = umin64(v, dpp_u64<0x141>(v));
  v = umin64(v, dpp_u64<0x140>(v));
  const uint64_t r0 = (uint64_t)readlane_i64((int64_t)v, 0);
  const uint64_t r1 = (uint64_t)readlane_i64((int64_t)v, 16);
  const uint64_t r2 = (uint64_t)readlane_i64((int64_t)v, 32);
  const uint64_t r3 = (uint64_t)readlane_i64((int64_t)v, 48);
  return umin64(umin64(r0, r1), umin64(r2, r3));
}

// The same for u32 with native DPP-fed v_min_u32.
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, dpp_u32<0xB1>(v));
  v = min(v, dpp_u32<0x4E>(v));
  v = min(v, dpp_u32<0x141>(v));
  v = min(v, dpp_u32<0x140>(v));
  const uint32_t r0 = readlane_u32(v, 0), r1 = readlane_u32(v, 16);
  const uint32_t r2 = readlane_u32(v, 32), r3 = readlane_u32(v, 48);
  return min(min(r0, r1), min(r2, r3));
}

// Sum over the 64 lanes (all active), every lane gets it.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += dpp_u32<0xB1>(v);
  v += dpp_u32<0x4E>(v);
  v += dpp_u32<0x141>(v);
  v += dpp_u32<0x140>(v);
  return readlane_u32(v, 0) + readlane_u32(v, 16) + readlane_u32(v, 32) + readlane_u32(v, 48);
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
  v += dpp_u64<0xB1>(v);
  v += dpp_u64<0x4E>(v);
  v += dpp_u64<0x141>(v);
  v += dpp_u64<0x140>(v);
  return (uint64_t)readlane_i64((int64_t)v, 0) + (uint64_t)readlane_i64((int64_t)v, 16) +
         (uint64_t)readlane_i64((int64_t)v, 32) + (uint64_t)readlane_i64((int64_t)v, 48);
}

// ---------------------------------------------------------------- Philox4x32-10

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const U4 n = {(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1,
                  (uint32_t)p0};
    c = n;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// -ln(u), u in (0, 1], using only IEEE +,-,*,/ so the host restatement
// (tests/tracegen.py::neg_log_unit) reproduces it bit for bit.
__device__ __forceinline__ double neg_log_unit(double u) {
#pragma clang fp contract(off)
  const uint64_t bits = (uint64_t)__double_as_longlong(u);
  int64_t e = (int64_t)((bits >> 52) & 0x7FF) - 1023;
  double m = __longlong_as_double((long long)((bits & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull));
  if (m > 1.4142135623730951) {
    m = m * 0.5;
    e = e + 1;
  }
  const double f = (m - 1.0) / (m + 1.0);
  const double f2 = f * f;
  double acc = 1.0 / 21.0;
  acc = acc * f2 + (1.0 / 19.0);
  acc = acc * f2 + (1.0 / 17.0);
  acc = acc * f2 + (1.0 / 15.0);
  acc = acc * f2 + (1.0 / 13.0);
  acc = acc * f2 + (1.0 / 11.0);
  acc = acc * f2 + (1.0 / 9.0);
  acc = acc * f2 + (1.0 / 7.0);
  acc = acc * f2 + (1.0 / 5.0);
  acc = acc * f2 + (1.0 / 3.0);
  acc = acc * f2 + 1.0;
  const double ln_m = 2.0 * f * acc;
  const double ln_u = (double)e * 0.6931471805599453 + ln_m;
  return -ln_u;
}

// ---------------------------------------------------------------- trace recipe
// The synthetic trace of one replication (tracegen.hip documents the recipe;
// tests/tracegen.py restates it on the host).  gen_kernel writes it to HBM;
// the replay kernels' generated mode (fognet_run_generated_dev) computes the
// same values 64 publishes at a time and never stores the trace.
struct GenRep {
  uint32_t k0, k1;  // Philox key (seed, global replication index)
  int32_t req_lo;
  uint32_t pad;
  uint64_t rspan;   // req_hi - req_lo + 1
  double mean;      // mean inter-arrival gap (ticks)
  int64_t scale;    // latency multiplier
};

// rl: local index into the per-replication parameter arrays
__device__ __forceinline__ GenRep gen_rep(const fognet_gen_params& p, int64_t r_global, int64_t rl) {
  GenRep g;
  g.k0 = p.seed;
  g.k1 = (uint32_t)r_global;
  g.req_lo = p.req_lo;
  g.pad = 0u;
  g.rspan = (uint64_t)(p.req_hi - p.req_lo) + 1ull;
  g.mean = p.mean_gap_ticks[rl];
  g.scale = p.lat_scale[rl];
  return g;
}

// node j: MIPS, downlink and uplink latency (its first advert arrives at init = ul)
__device__ __forceinline__ void gen_node(const GenRep& g, int j, int32_t& m, int64_t& d, int64_t& u) {
  const uint64_t span = 1000000000ull - 1000000ull + 1ull;
  const U4 x = philox4x32_10(U4{(uint32_t)j, 1u, 0u, 0u}, g.k0, g.k1);
  d = (int64_t)(1000000ull + (uint64_t)x.x % span) * g.scale;
  u = (int64_t)(1000000ull + (uint64_t)x.y % span) * g.scale;
  m = 1000 * (1 + j % 4);
}

// task i: requirement and the gap before it (arrive[i] = arrive[i-1] + gap,
// arrive[-1] = max_j ul_j + 1)
__device__ __forceinline__ void gen_task(const GenRep& g, int i, int64_t& gap, int32_t& rq) {
  const U4 x = philox4x32_10(U4{(uint32_t)i, 0u, 0u, 0u}, g.k0, g.k1);
  rq = (int32_t)((uint64_t)g.req_lo + (uint64_t)x.x % g.rspan);
  const uint64_t k53 = ((uint64_t)x.y << 21) | ((uint64_t)x.z >> 11);
  const double u = (double)(k53 + 1ull) * 0x1p-53;
  gap = (int64_t)(g.mean * neg_log_unit(u));
}

// ---------------------------------------------------------------- replay

// Pending-task ring entry of the register kernel (replay.hip): one 8-B word
// per task assigned to a node, kept until the advertisement of its
// completion has been applied to the broker's view:
//   bits 8..63  arrival tick at the node (broker decision tick + dl), < 2^56
//   bits 0..7   service seconds, requiredMIPS / MIPS (int division), < 2^8
// The cumulative service of an entry is not stored: it follows from the
// head's (+ S) or the tail's (- the later entries' S).  Two consecutive
// entries share a 16-B aligned pair, which the head+1 prefetch loads at once,
// so one cache-line fetch serves two completions.  A task outside these
// ranges (a simulated time past 2^56 ticks = 20 h, or a service time above
// 255 s) hands its replication to the wide kernel (exact, unbounded).
typedef uint64_t RingWord;
constexpr int kRingSBits = 8;
constexpr uint32_t kRingSMask = (1u << kRingSBits) - 1u;
constexpr int64_t kRingAMax = (int64_t)((1ull << (64 - kRingSBits)) - 1ull);

struct ReplayArgs {
  int32_t R, T, N, node_stride;
  int32_t q_log2;  // ring capacity per node = 1 << q_log2
  uint32_t max_s;  // largest admissible service time (keeps busy < 2^32)
  int32_t policy;  // fognet_policy
  int32_t fuse_stats;  // 1: replay_kernel also computes the statistics pass (rep_stats) as an epilogue
  const int64_t* arrive;
  const int32_t* req;
  const int32_t* mips;
  const int64_t* dl;
  const int64_t* ul;
  const int64_t* init;
  int32_t* out_node;
  uint8_t* out_status;
  int64_t* out_start;
  int64_t* out_done;
  fognet_rep_stats* out_stats;
  RingWord* ring;  // [R][N][Q]
  const double* p_busy;   // [R|1][N] power model (nullable)
  const double* p_idle;
  double* out_energy;     // [R][N] (nullable)
  int64_t* hist;          // [FOGNET_HIST_METRICS][FOGNET_HIST_BINS], added to (nullable)
  const int64_t* down;    // [R|1][N] node crash ticks (nullable; wide kernel only)
  // Replications the register kernel hands to the wide kernel (a node past the
  // ring capacity, or a service time past max_s): the register kernel appends
  // r to wide_list (wide_count: device counter, zeroed before it); the wide
  // kernel, launched with wide_list set, replays exactly the listed ones.
  int32_t* wide_list;     // [R] (nullable: no hand-over, kNeedsWide stays the status)
  int32_t* wide_count;
  // Statistics-only replays (fognet_batch_out per-task arrays null): the wide
  // kernel, which accumulates its statistics inline, then writes nothing per
  // task; the register kernel writes to an internal [R][T] scratch instead
  // (its fused statistics epilogue reads the outputs back).
  int32_t no_task_out;
  // FOGNET_POLICY_EXT_HIER (wide kernel): [R][T] regional broker per publish, escalation
  // threshold (advertised busy seconds) and the escalated task's extra latency
  const int32_t* region;
  int64_t hier_up;
  int32_t hier_thr;
  // Generated mode (fognet_run_generated_dev): gen_on != 0 ->
  // replication r's trace and node parameters are the gen_kernel recipe's for
  // global index gen_r0 + r, computed in the kernel (arrive/req/mips/dl/ul/init
  // unused), and only statistics are written (no per-task outputs).
  // 1: replay_inl_kernel (statistics accumulated in the loop, no epilogue
  // re-read; fused-statistics replays while T * max_s < 2^32)
  int32_t inloop;
  int32_t gen_on;
  int32_t gen_slots;  // generated mode: workgroups (and ring slots) of the work-counter launch
  int64_t gen_r0;
  fognet_gen_params gen;
  int32_t* queue;     // generated mode: work counter (zeroed before the launch)
  // replay_kernel's progress board (kBoardWords u32, 0xFF-filled before the
  // launch): one word per hardware wave slot (XCC, SE, SH, CU, SIMD, wave),
  // the wave's replay progress, read by the other waves of its SIMD to set
  // their issue priority (least progress first).  Nullable.
  uint32_t* board;
  // FOGNET_FLAG_REF_ABORT: a replication with an abort point gets status FOGNET_REF_ABORTED
  int32_t ref_abort;
};
constexpr size_t kBoardWords = (size_t)1 << 17;  // 8 XCC x 8 SE x 2 SH x 16 CU x 4 SIMD x 16 slots

// Generated-mode launch: 3 waves per SIMD, 4 SIMDs per CU (replay_gen_kernel)
constexpr int kGenWavesPerCu = 12;

// Internal per-replication status between the two replay kernels (never
// returned: the wide kernel overwrites the record of every listed replication).
constexpr int32_t kNeedsWide = 0x57494445;

// FOGNET_HIST_BINS rule (fognet_hip.h): whole milliseconds, log2 bins.
// Bit length of q = ticks / 1e9 without the 64-bit division: with L the bit
// length of ticks, 1e9 * 2^j (bit length 30 + j) is below ticks for every
// j < L - 30 and the one j = L - 30 takes a compare.
__device__ __forceinline__ int hist_bin(int64_t ticks) {
  if (ticks < 1000000000ll) return 0;
  const int j = 34 - __clzll((long long)ticks);  // L - 30 >= 0
  const int b = j + ((uint64_t)ticks >= (1000000000ull << j) ? 1 : 0);
  return b > FOGNET_HIST_BINS - 1 ? FOGNET_HIST_BINS - 1 : b;
}

// Wide replay (replay_wide.hip, N > 256): the pending-task chain of a node is
// linked through per-task entries instead of a fixed per-node ring.
struct WideEntry {
  int64_t a;     // arrival tick at the node
  int64_t done;  // completion (RELEASERESOURCE) tick
  uint64_t C;    // cumulative service seconds assigned to the node, this task included
  uint32_t S;    // service seconds, requiredMIPS / MIPS (int division)
  int32_t prev;  // previous task on the same node (-1: none)
  int32_t next;  // next task on the same node (valid while this one is pending)
  int32_t pad;   // 1: escalated to the parent broker (FOGNET_POLICY_EXT_HIER)
};
static_assert(sizeof(WideEntry) == 40, "wide entry is 40 B");

// Per node: chain ends plus copies of the head's and tail's fields, so a push
// or an advert starts from one 64-B record (one cache line) instead of
// chasing entries.  The `next` of the head lives here (hd_next); the `next` of
// every other pending task in its WideEntry.
struct WideNode {
  int32_t hd, tl;   // oldest pending / newest task of the node (-1: none yet)
  int32_t npend;    // tasks whose completion advert has not reached the broker
  int32_t hd_next;  // task after the head (valid while npend >= 2)
  int64_t hd_done;  // head: completion tick
  uint64_t hd_C;    //       cumulative service
  int64_t tl_a;     // tail: arrival tick
  int64_t tl_done;  //       completion tick
  uint64_t tl_C;    //       cumulative service (0: no task yet) = the node's service seconds so far
  uint32_t hd_S, tl_S;  // (bit 31 of tl_S: the tail was escalated, FOGNET_POLICY_EXT_HIER)
};
static_assert(sizeof(WideNode) == 64, "wide node record is one 64-B line");

// LDS of the wide kernel: per lane and group of 16 of its nodes the earliest
// advert, its node, the smallest view key and run-horizon bound (28 B) + the histogram; the
// per-node view (next advert tick, advertised busy) is in HBM.
constexpr int kWideGroupSlots = 16;
constexpr int kWideMaxNodes = 65536;  // LDS: 115 KiB of group minima (FOGNET_POLICY_EXT_HIER's limit)
// Above kWideMaxNodes the flat policies keep the group minima in HBM (2 KiB per group of
// 1,024 nodes per workspace slot), up to:
constexpr int kWideBigMaxNodes = 1 << 20;
size_t replay_wide_lds_bytes(int32_t N);
// workspace: R*T WideEntry followed by R*N WideNode
// (+ R*N generated node parameters in generated mode, + the HBM group minima above kWideMaxNodes)
size_t replay_wide_workspace_bytes(int32_t R, int32_t T, int32_t N, bool gen, int policy);
// FOGNET_POLICY_EXT_HIER by region (replay_region.hip): one wavefront per
// (replication, region) over the region's publishes while no escalation occurs;
// then per replication the regions' records merged and the statistics pass, or
// the replication appended to a.wide_list for the sequential wide kernel.
struct RegionRec {
  int32_t n_done, max_pend, status, pad;
};
struct RegionWs {
  WideEntry* e;    // [R][T] chain entries, indexed by the task's position in the region-sorted order
  WideNode* nd;    // [R][N]
  RegionRec* rec;  // [R][B]
  uint32_t* vb;    // [R][B][16][64] advertised busy times (the region kernel's view, [slot][lane])
  // [R] the replication's first escalated publish (trace index), lowered by every region that meets
  // one (atomic min); set to T by the sort kernel, 0 for anything the sequential kernel must replay
  // from the start (an invalid trace, a saturated view, a service time past the pass's range).  A
  // region wavefront of the first pass stops once its publishes are past it.
  int32_t* esc;
  int32_t* s_idx;  // [R][T] trace index of sorted position p (inv's inverse)
  unsigned char* pacc;  // [R][kRegionResumeBytes] the statistics of the publishes before esc (finish kernel)
  // 1: every replication, up to its first escalation (found on the way); 2: the escalated
  // replications again, each region exactly up to esc (a first-pass wavefront may have run past
  // it), so that the sequential wide kernel continues from that state (resume)
  int32_t pass;
  int32_t* seg;    // [R][B + 1] region b's publishes are sorted positions [seg[b], seg[b + 1])
  int64_t* s_arr;  // [R][T] publish ticks, region-sorted (stable: trace order within a region)
  int32_t* s_req;  // [R][T] MIPSRequired, region-sorted
  int32_t* inv;    // [R][T] sorted position of task i
  int32_t* o_node;   // [R][T] the region pass's per-task outputs, region-sorted (region_finish_kernel
  uint8_t* o_status; //        writes them to the caller's arrays in trace order)
  int64_t* o_start;
  int64_t* o_done;
  int64_t* tails;  // [R][N][2] every node's tail completion tick (INT64_MIN: no task) and service seconds (tl_C):
                   // written at the region pass's start, at each write-back of a lane's cached record and at its
                   // end, so the finish kernel reads 16 B per node instead of the 64-B records
  uint32_t* okey;  // [R][B] dispatch key of each (replication, region): estimated load, quantised (region_sort_kernel)
  int32_t* perm;   // [R * B] the region wavefronts' dispatch order: lightest estimated load first (region_order_kernel)
  int32_t B;       // regions: ceil(N / FOGNET_HIER_REGION_NODES)
};
// sort + order + the first region pass; resume: + the second pass over the escalated replications;
// then the finish kernel (statistics, hand-over list)
hipError_t launch_replay_region(const ReplayArgs& a, const RegionWs& w, bool resume, hipStream_t s);
constexpr size_t kRegionResumeBytes = 192;  // >= sizeof(Acc) + sizeof(AbortPt) (replay_common.h)

// slots: workspace slots (workgroups).  With a.wide_list unset, slots == R and
// workgroup r replays replication r; with it set, the workgroups take the
// listed replications in turn (slots <= R bounds the workspace).  rw (EXT_HIER,
// nullable): the region pass's workspace; a listed replication with 0 < rw->esc[r] < T
// continues from the second pass's state at its first escalated publish.
hipError_t launch_replay_wide(const ReplayArgs& a, void* workspace, int32_t slots, hipStream_t s,
                              const RegionWs* rw = nullptr);

hipError_t launch_replay(const ReplayArgs& a, hipStream_t s);
hipError_t launch_rep_stats(const ReplayArgs& a, hipStream_t s);
// Job reduction: one block up to kReduceChunk records, else blocks of
// kReduceChunk into reduce_stats_parts(R) partial records (workspace `parts`)
// and a merge.
constexpr int32_t kReduceChunk = 4096;
int32_t reduce_stats_parts(int32_t R);
hipError_t launch_reduce_stats(const fognet_rep_stats* st, int32_t R, fognet_job_stats* out, fognet_job_stats* parts,
                               hipStream_t s);
hipError_t launch_decide(int64_t m, int32_t n, int64_t view_stride, const double* busy, const int32_t* mips,
                         const int32_t* req, int32_t* node, int32_t* status, hipStream_t s);
// fognet_decide's kernel arguments: the view of up to kDecideArgNodes nodes by value
constexpr int kDecideArgNodes = 256;
struct DecideArgs {
  int32_t n, mips0, req, pad;
  double busy[kDecideArgNodes];
};
hipError_t launch_decide_args(const DecideArgs& a, const double* far_busy, int32_t* res, hipStream_t s);
hipError_t launch_decide_v2(int64_t m, int32_t n, const int32_t* mips, const int32_t* local, const int32_t* req,
                            int32_t* node, int32_t* action, hipStream_t s);
hipError_t launch_user_stats(const ReplayArgs& a, const int64_t* user_ul, const int64_t* user_dl, int32_t per_task,
                             fognet_user_stats* out, hipStream_t s);
// v2 model replay (replay_v2.hip)
size_t replay_v2_workspace_bytes(int32_t R, int32_t T, int32_t N, int32_t q_log2);
hipError_t launch_replay_v2(const fognet_v2_in& in, const fognet_v2_out& out, void* workspace, int32_t q_log2,
                            hipStream_t s);
hipError_t launch_gen_trace(const fognet_gen_params& p, int64_t r0, int32_t R, int32_t T, int32_t N,
                            int64_t* arrive, int32_t* req, int32_t* mips, int64_t* dl, int64_t* ul,
                            int64_t* init, hipStream_t s);

}  // namespace fognet
