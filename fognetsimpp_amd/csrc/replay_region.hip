// replay_region.hip — FOGNET_POLICY_EXT_HIER replayed one regional broker per
// wavefront (BASELINE.json configs[4], C5: 10 regions of 1,024 fog nodes).
//
// Under EXT_HIER a publish goes to its region's broker, which chooses the
// smallest (advertised busy, index) of its own region (BrokerBaseApp3.cc:
// 265-304 restricted to the region) and escalates to the parent only when that
// busy time exceeds the threshold (fognet_hip.h).  Until the first escalation
// of a replication its regions are therefore independent: a region's view
// changes only at adverts of its own nodes (BrokerBaseApp3.cc:123-130), whose
// busy values depend only on the tasks its own broker sent them
// (ComputeBrokerApp3.cc:224-320).  So each (replication, region) pair is
// replayed by its own wavefront over the region's publishes only:
//   * region_sort_kernel (one 256-thread block per replication) sorts the
//     publishes by region, stably (a counting sort), so region b's publishes
//     are the contiguous positions [seg[b], seg[b+1]) of a sorted copy of the
//     trace, and checks the trace's preconditions once;
//   * replay_region_kernel walks its region's segment 64 publishes at a time
//     with the flat wide kernel's closed form and decision runs (replay_wide.hip,
//     DESIGN.md §3.6): due adverts applied lane-parallel, the regional minimum
//     key, then every publish up to the run horizon E pushed onto the chosen
//     node with one FIFO scan.  Node l of the region (index base + l) lives on
//     lane l % 64, slot l / 64: next-advert ticks and run-horizon offsets in
//     LDS, advertised busy times in HBM, records and task chains in HBM, the
//     lane's last-pushed record cached in registers;
//   * region_finish_kernel merges the regions' records, writes the outputs back
//     in trace order and runs the statistics pass (the same Acc record,
//     histogram and a11 energy as the wide kernel's inline statistics).
// A replication in which a region meets an escalation is continued by the
// sequential wide kernel from the publish that escalates (resume): the first
// pass finds each replication's first escalated publish (every region stops once
// its publishes are past the earliest found so far), a second pass replays the
// escalated replications again with each region stopping exactly before it (a
// first-pass wavefront may have run past it), the finish kernel completes the
// publishes before it, and the wide kernel takes over that state (its node
// records, chains and views, replay_wide.hip).  Anything else this pass does not
// model (a saturated busy time, a service time past 2^22 s, an invalid input)
// hands the replication to the wide kernel from the start, as does
// FOGNET_HIER_RESUME=0 for every escalated one.
#include "replay_common.h"

namespace fognet {

namespace {

constexpr int kRegionSlots = FOGNET_HIER_REGION_NODES / kWave;  // 16 view slots per lane
static_assert(kRegionSlots == kWideGroupSlots, "a region is one wide-kernel group row");
constexpr uint32_t kRegBusySat = 0xFFFFFFFFu;
constexpr uint32_t kRegSCap = 1u << 22;  // the wide kernel's kWideSCap: past it the sequential kernel decides
// Run-horizon offsets are capped (replay_wide.hip's node_w caps at 2^21 s): a smaller offset only
// shortens runs.  16 bits here, so the view ticks and offsets take 10 KiB of LDS per wavefront and
// 16 wavefronts fit per CU (12 KiB with 32-bit offsets: 13); C5's offsets are minutes at most.
constexpr uint32_t kRegWCap = 0xFFFFu;

// Internal per-(replication, region) status: replay the replication sequentially
// (fognet_hip.h never returns it; under FOGNET_HIER_REGIONS=only the finish kernel
// reports FOGNET_ERR_UNSUPPORTED instead).
constexpr int32_t kRegionSeq = 0x53455121;
constexpr int kQuitEvery = 4;  // chunks between polls of the replication's first escalation (W.esc)

// ---- region_sort_kernel: stable counting sort of one replication's publishes by region (one block)
constexpr int kSortThreads = 1024;  // (a replication's 10,000 publishes in 10 tiles)
constexpr int kSortWaves = kSortThreads / kWave;

__global__ __launch_bounds__(kSortThreads) void region_sort_kernel(ReplayArgs A, RegionWs W) {
  const int r = blockIdx.x, tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const int T = A.T, B = W.B;
  const size_t tbase = (size_t)r * (size_t)T;
  __shared__ uint32_t s_cnt[kWave];             // per region: count, then the next free position
  __shared__ uint32_t s_wc[kSortWaves][kWave];  // per wave and region: the tile's publishes
  __shared__ int s_bad;
  // the dispatch key's inputs: the replication's requirement and MIPS totals (per-wave partials),
  // each region's first sorted position
  __shared__ unsigned long long s_rq[kSortWaves], s_mp[kSortWaves];
  __shared__ uint32_t s_seg[kWave + 1];
  if (tid < kWave) s_cnt[tid] = 0u;
  if (tid == 0) s_bad = 0;
  __syncthreads();
  // counts, and the trace preconditions the sequential kernel reports (nondecreasing ticks,
  // requirement >= 0, ticks < 2^61, a region of the node set): a violation hands r over
  bool bad = false;
  uint64_t rq = 0u, mp = 0u;
  for (int i = tid; i < T; i += kSortThreads) {
    const int32_t g = A.region[tbase + i];
    const int64_t t = A.arrive[tbase + i];
    const int64_t tp = i > 0 ? A.arrive[tbase + i - 1] : INT64_MIN;
    const int32_t q = A.req[tbase + i];
    if (g < 0 || g >= B || q < 0 || t > kMaxTick || t < tp) {
      bad = true;
    } else {
      atomicAdd(&s_cnt[g], 1u);
      rq += (uint32_t)q;
    }
  }
  for (int j = tid; j < A.N; j += kSortThreads) {
    const int32_t m = A.mips[(size_t)r * (size_t)A.node_stride + j];
    mp += (uint32_t)(m > 0 ? m : 1);
  }
  rq = wave_sum_u64(rq);
  mp = wave_sum_u64(mp);
  if (lane == 0) {
    s_rq[wv] = rq;
    s_mp[wv] = mp;
  }
  if (bad) s_bad = 1;
  __syncthreads();
  int32_t* const seg = W.seg + (size_t)r * (size_t)(B + 1);
  // (no escalation found yet; an invalid trace: the sequential kernel replays r from the start)
  if (tid == 0) __hip_atomic_store(W.esc + r, s_bad ? 0 : T, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (s_bad) {
    // the dispatch inputs stay defined: empty segments, dispatched last
    if (tid <= B) seg[tid] = 0;
    if (tid < B) W.okey[(size_t)r * B + tid] = 255u;
    return;
  }
  if (tid == 0) {
    uint32_t acc = 0u;
    for (int b = 0; b < B; ++b) {
      const uint32_t c = s_cnt[b];
      s_cnt[b] = acc;
      seg[b] = (int32_t)acc;
      s_seg[b] = acc;
      acc += c;
    }
    seg[B] = (int32_t)acc;
    s_seg[B] = acc;
  }
  // tiles of kSortThreads publishes: a publish's position = its region's next free position + the
  // publishes of its region in earlier waves of the tile + those in earlier lanes of its wave
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int i0 = 0; i0 < T; i0 += kSortThreads) {
    s_wc[wv][lane] = 0u;
    __syncthreads();
    const int i = i0 + tid;
    const bool live = i < T;
    const int32_t g = live ? A.region[tbase + i] : -1;
    uint32_t rank = 0u;
    for (uint64_t rem = ballot(live); rem;) {
      const int g0 = __builtin_amdgcn_readlane(g, (int)__builtin_ctzll(rem));
      const uint64_t m = ballot(live && g == g0);
      if (live && g == g0) rank = (uint32_t)__popcll(m & lt);
      if (lane == 0) s_wc[wv][g0] = (uint32_t)__popcll(m);
      rem &= ~m;
    }
    __syncthreads();
    if (live) {
      uint32_t pos = s_cnt[g] + rank;
      for (int w = 0; w < wv; ++w) pos += s_wc[w][g];
      W.inv[tbase + i] = (int32_t)pos;
      W.s_idx[tbase + pos] = i;
      W.s_arr[tbase + pos] = A.arrive[tbase + i];
      W.s_req[tbase + pos] = A.req[tbase + i];
    }
    __syncthreads();
    if (tid < B) {
      uint32_t c = 0u;
      for (int w = 0; w < kSortWaves; ++w) c += s_wc[w][tid];
      s_cnt[tid] += c;
    }
    __syncthreads();
  }
  if (tid < B) {
    // dispatch key: the region's estimated load, rho = (its publishes x the replication's mean
    // service seconds) over (its span x its nodes), from its first and last sorted publish; a
    // lighter region decides in more, shorter runs (one per publish at the lightest), so its
    // wavefront runs longer: the region wavefronts are dispatched lightest first
    // (region_order_kernel), i.e. longest first.  Only the schedule changes, never a result.
    const int nb = min(FOGNET_HIER_REGION_NODES, A.N - tid * FOGNET_HIER_REGION_NODES);
    const uint32_t p0 = s_seg[tid], n = s_seg[tid + 1] - p0;
    uint32_t key = 255u;  // (no publish: last)
    if (n > 0u) {
      uint64_t rqt = 0u, mpt = 0u;
      for (int w = 0; w < kSortWaves; ++w) {
        rqt += s_rq[w];
        mpt += s_mp[w];
      }
      const double svc = ((double)rqt / (double)(T > 0 ? T : 1)) / ((double)mpt / (double)A.N);
      const double span = (double)(W.s_arr[tbase + p0 + n - 1] - W.s_arr[tbase + p0]) * 1e-12 + 1e-3;
      const double rho = (double)n * svc / (span * (double)nb);
      const double q = 8.0 * log2(rho > 1e-30 ? rho : 1e-30) + 128.0;
      key = (uint32_t)(q < 0.0 ? 0.0 : (q > 254.0 ? 254.0 : q));
    }
    W.okey[(size_t)r * B + tid] = key;
  }
}

// ---- region_order_kernel: the region wavefronts' dispatch order, by key (one block; counting
// sort, any order within a key)
constexpr int kOrderThreads = 1024;
__global__ __launch_bounds__(kOrderThreads) void region_order_kernel(int32_t n, RegionWs W) {
  __shared__ uint32_t s_h[256];
  const int tid = threadIdx.x;
  if (tid < 256) s_h[tid] = 0u;
  __syncthreads();
  for (int i = tid; i < n; i += kOrderThreads) atomicAdd(&s_h[W.okey[i] & 255u], 1u);
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = 0u;
    for (int k = 0; k < 256; ++k) {
      const uint32_t c = s_h[k];
      s_h[k] = acc;
      acc += c;
    }
  }
  __syncthreads();
  for (int i = tid; i < n; i += kOrderThreads) W.perm[atomicAdd(&s_h[W.okey[i] & 255u], 1u)] = i;
}

// ---- replay_region_kernel
// Run horizon offset of a node (replay.hip horizon_all_in): with every pending
// task arrived before its head completes, the node's next advert carries
// v1 = tl_C - hd_C and each later one falls by at most the seconds elapsed, so an
// advert with busy <= thr comes no earlier than nxt + (v1 - thr) s.  The offset
// v1 (capped: a smaller one only shortens runs) is kept per slot; tasks still in
// flight: offset 0 (the bound is then the next advert itself).
__device__ __forceinline__ uint32_t w_offset(const WideNode& h, int64_t dl) {
  if (h.npend == 0 || !arrives_before(h.tl_a, h.hd_done, dl, h.hd_S)) return 0u;
  const uint64_t v1 = h.tl_C - h.hd_C;
  return v1 < (uint64_t)kRegWCap ? (uint32_t)v1 : kRegWCap;
}

// 4 waves per SIMD (<= 128 VGPRs); 10 KiB of LDS per wavefront (view ticks and horizon offsets).
// PASS 1: every replication, up to its first escalation; 2: the escalated ones again, exactly up
// to it (RegionWs::pass; two instantiations, so kernel traces tell the passes apart).
template <int PASS>
__global__ __launch_bounds__(64, 4) void replay_region_kernel(ReplayArgs A, RegionWs W) {
  const int B = W.B;
  const int item = W.perm[blockIdx.x];  // (region_order_kernel's dispatch order)
  const int r = item / B, b = item - (item / B) * B;
  const int rb = r * B + b;  // (r, b)'s region record and busy view
  const int lane = threadIdx.x;
  const int T = A.T, N = A.N;
  const int base = b * FOGNET_HIER_REGION_NODES;
  const int nb = min(FOGNET_HIER_REGION_NODES, N - base);  // nodes of this region (>= 1)
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  WideEntry* const e = W.e + tbase;  // indexed by sorted position
  WideNode* const nd = W.nd + (size_t)r * (size_t)N;
  int64_t* const tails = W.tails + 2 * (size_t)r * (size_t)N;
  // node j's tail (completion, service seconds) for the finish kernel: a node's tail changes only
  // when a run is pushed onto it, i.e. while it is a lane's cached node
  auto write_tail = [&](int j, const WideNode& h) {
    tails[2 * (size_t)j] = h.tl >= 0 ? h.tl_done : INT64_MIN;
    tails[2 * (size_t)j + 1] = (int64_t)h.tl_C;
  };
  const int32_t* const seg = W.seg + (size_t)r * (size_t)(B + 1);
  const int64_t arrive0 = T > 0 ? A.arrive[tbase] : kNever;
  const int32_t esc0 = __hip_atomic_load(W.esc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the second pass replays only the replications the first found an escalation in (0 < esc < T);
  // the others keep the first pass's state and records
  if (PASS == 2 && (esc0 <= 0 || esc0 >= T)) return;
  // esc 0: an invalid trace (see the sort) or another region's failure: the sequential kernel replays r
  uint32_t err = esc0 == 0 ? (uint32_t)kRegionSeq : (uint32_t)FOGNET_OK;
  const int s0 = err == FOGNET_OK ? seg[b] : 0;
  int nseg = err == FOGNET_OK ? seg[b + 1] - s0 : 0;  // this region's publishes
  if (PASS == 2) {  // those before the escalated publish: a prefix of the segment (trace order)
    int lo = 0, hi = nseg;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (W.s_idx[tbase + s0 + mid] < esc0) lo = mid + 1;
      else hi = mid;
    }
    nseg = lo;
  }
  // the first pass's finding for W.esc: the escalated publish's trace index, 0 for a failure the
  // sequential kernel must replay from the start, -1 none (or a stop at another region's escalation)
  int32_t esc_hit = -1;

  // ---- this lane's nodes (local l = s * 64 + lane) and their view ([slot][lane]: each lane
  // touches only its own column): next advert ticks and run-horizon offsets in LDS
  // (conflict-free); advertised busy times in HBM (RegionWs::vb; read back only by a key
  // rescan of a lane without a zero-busy slot)
  __shared__ int64_t s_nxt[kRegionSlots * kWave];
  __shared__ uint16_t s_woff[kRegionSlots * kWave];
  int64_t* const vnxt = s_nxt + lane;  // vnxt[s * kWave]: slot s of this lane
  uint16_t* const vwoff = s_woff + lane;
  uint32_t* const vbusy = W.vb + (size_t)rb * (size_t)(kRegionSlots * kWave) + lane;
  bool bad = false;
  // slots with an advert pending (view tick not kNever) and slots whose advertised busy
  // time is not 0, as bit masks: the rescans below visit only the first kind, and a
  // lane with a zero-busy slot has its smallest key without reading the view
  uint32_t act = 0u, nzb = 0u;
#pragma unroll
  for (int s = 0; s < kRegionSlots; ++s) {
    const int l = s * kWave + lane;
    vnxt[s * kWave] = kNever;
    vwoff[s * kWave] = 0u;
    vbusy[s * kWave] = l < nb ? 0u : kRegBusySat;  // (past the region: never the minimum)
    nzb |= l < nb ? 0u : 1u << s;
    if (l < nb) {
      const int j = base + l;
      const int32_t m = A.mips[nbase + j];
      const int64_t d = A.dl[nbase + j], u = A.ul[nbase + j], ia = A.init[nbase + j];
      bad |= (m <= 0) | (d < 0) | (u < 0) | (d > kMaxTick) | (u > kMaxTick) | (ia < u) | (ia >= arrive0);
      nd[j] = WideNode{-1, -1, 0, -1, 0, 0u, 0, 0, 0u, 0u, 0u};
      tails[2 * (size_t)j] = INT64_MIN;  // (no task yet)
      tails[2 * (size_t)j + 1] = 0;
    }
  }
  // the lane's earliest advert (slot ms) and smallest view key (busy << 32 | j)
  int64_t mn = kNever;
  int ms = 0;
  uint64_t mk = lane < nb ? (uint64_t)(uint32_t)(base + lane) : ~0ull;
  // earliest advert over the pending slots (ties: the smallest slot)
  auto rescan_nxt = [&]() {
    mn = kNever;
    ms = 0;
    for (uint32_t m = act; m; m &= m - 1u) {
      const int s = __builtin_ctz(m);
      const int64_t x = vnxt[s * kWave];
      if (x < mn) {
        mn = x;
        ms = s;
      }
    }
  };
  // (partially unrolled: a full unroll issues all 16 loads at once and holds 32 VGPRs)
  auto rescan_key = [&]() {
    const uint32_t z = ~nzb & ((1u << kRegionSlots) - 1u);
    if (z) {  // a zero-busy slot: the smallest one holds the smallest key
      mk = (uint32_t)(base + __builtin_ctz(z) * kWave + lane);
      return;
    }
    mk = ~0ull;
#pragma unroll 1
    for (int q0 = 0; q0 < kRegionSlots; q0 += 8) {  // (8 loads in flight: few registers)
      uint32_t bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) bv[u] = vbusy[(q0 + u) * kWave];
      sync_vm();  // (in this arm: see sync_vm)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint64_t key = ((uint64_t)bv[u] << 32) | (uint32_t)(base + (q0 + u) * kWave + lane);
        mk = key < mk ? key : mk;
      }
    }
  };

  if (ballot(bad)) {
    err = kRegionSeq;
    esc_hit = 0;
  }
  uint32_t max_pend = 0u;
  int n_done = 0;
  // the node this lane pushed to last (the stale view keeps choosing it): its
  // record and parameters in registers, written back when the lane pushes to
  // another node and at the end (replay_wide.hip's cache)
  int cj = -1;
  WideNode ch{};
  UDiv c_dv{1u, 0u};
  int64_t c_dl = 0, c_ul = 0;
  auto cache_node = [&](uint32_t kk, int kl) {
    if (lane == kl && (int)kk != cj) {
      if (cj >= 0) {
        nd[cj] = ch;
        write_tail(cj, ch);
      }
      cj = (int)kk;
      ch = nd[kk];
      c_dv = udiv_magic((uint32_t)A.mips[nbase + kk]);
      c_dl = A.dl[nbase + kk];
      c_ul = A.ul[nbase + kk];
      sync_vm();  // (here: a hit then waits for nothing)
    }
  };
  bool view_changed = true;
  uint64_t key = 0ull;  // the regional broker's choice: its smallest view key
  // a run that used up its chunk continues in the next one while the publishes stay
  // within its horizon E_carry (the decision unchanged: no advert can change it before)
  bool carry = false;
  int64_t E_carry = 0;
  const int64_t* const sa = W.s_arr + tbase + s0;
  const int32_t* const sq = W.s_req + tbase + s0;
#ifdef FOGNET_REGION_PROF
  // profile build only: loop counters and clock64 segments, printed for a few wavefronts
  uint64_t pr[12] = {};
  uint64_t pt = clock64();
  const uint64_t pt0 = pt;
#define PRC(i, v) pr[i] += (v)
#define PRT(i) { const uint64_t _n = clock64(); pr[i] += _n - pt; pt = _n; }
#else
#define PRC(i, v)
#define PRT(i)
#endif

  for (int c0 = 0; c0 < nseg && err == FOGNET_OK; c0 += kWave) {
    // first pass: this region's publishes are past r's first escalation found so far (another
    // region's, or 0 for a failure), so nothing it decides from here on matters
    if (PASS == 1 && (c0 & (kQuitEvery * kWave - 1)) == 0 && c0 > 0 &&
        W.s_idx[tbase + s0 + c0] >= __hip_atomic_load(W.esc + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
      err = kRegionSeq;
      break;
    }
    const int cnt = min(kWave, nseg - c0);
    const bool live = lane < cnt;
    const int64_t ca = live ? sa[c0 + lane] : kNever;
    const int32_t cr = live ? sq[c0 + lane] : 0;
    // this chunk's pushed tasks, one per lane (sorted position s0 + c0 + lane): outputs
    // stored once per chunk, coalesced
    bool q_on = false;
    uint32_t q_k = 0u, q_status = 0u;
    int64_t q_start = 0, q_done = 0;
    int jp = 0;
    while (jp < cnt) {
      const int64_t t = readlane_i64(ca, jp);
      const bool resume = carry && t <= E_carry;
      carry = false;
      int64_t E = E_carry;
      PRC(0, 1);
      PRC(1, resume ? 1 : 0);
      PRT(7)
      if (!resume) {
        // 1) completion adverts that reached the broker strictly before t, lane-parallel
        bool lbroken = false;
        if (ballot(mn < t)) view_changed = true;
        while (ballot(mn < t)) {
          PRC(2, 1);
          PRC(3, __popcll(ballot(mn < t)));
          PRC(4, __popcll(ballot(mn < t && base + ms * kWave + lane == cj)));
          if (mn < t) {
            const int sl = ms;
            const int j = base + sl * kWave + lane;
            const bool hit = j == cj;
            int64_t nxt_j;
            uint32_t busy_j, off_j;
            bool broken = false;
            // the node's adverts that are due, in order; the cached record is updated in place
            if (hit) {
              (void)apply_wide_advert(ch, e, c_dl, c_ul, 0, nxt_j, busy_j, broken);
              while (nxt_j < t && !broken) (void)apply_wide_advert(ch, e, c_dl, c_ul, 0, nxt_j, busy_j, broken);
              off_j = w_offset(ch, c_dl);
            } else {  // (waited for here, not where the arms meet: sync_vm)
              WideNode h = nd[j];
              const int64_t dl_j = A.dl[nbase + j], ul_j = A.ul[nbase + j];
              sync_vm();
              (void)apply_wide_advert(h, e, dl_j, ul_j, 0, nxt_j, busy_j, broken);
              while (nxt_j < t && !broken) (void)apply_wide_advert(h, e, dl_j, ul_j, 0, nxt_j, busy_j, broken);
              off_j = w_offset(h, dl_j);
              nd[j] = h;
            }
            lbroken |= broken;
            vnxt[sl * kWave] = nxt_j;
            vwoff[sl * kWave] = (uint16_t)off_j;
            vbusy[sl * kWave] = busy_j;
            act = nxt_j != kNever ? act | (1u << sl) : act & ~(1u << sl);
            nzb = busy_j != 0u ? nzb | (1u << sl) : nzb & ~(1u << sl);
            rescan_nxt();
            // the key: only j's changed; a rescan only when j held the minimum and grew
            const uint64_t nk = ((uint64_t)busy_j << 32) | (uint32_t)j;
            if ((uint32_t)mk == (uint32_t)j && nk > mk) rescan_key();
            else mk = nk < mk ? nk : mk;
          }
        }
        if (ballot(lbroken)) {
          err = FOGNET_ERR_INTERNAL;
          esc_hit = 0;
          break;
        }
        PRT(8)
        // 2) the regional broker's decision; above the threshold it would escalate
        if (view_changed) {
          key = wave_min_u64(mk);
          view_changed = false;
        }
        if ((key >> 32) > (uint64_t)A.hier_thr || (key >> 32) >= kRegBusySat) {
          err = kRegionSeq;
          // an escalation (publish s0 + c0 + jp), or a saturated view (the sequential kernel refuses it)
          esc_hit = (key >> 32) >= kRegBusySat ? 0 : W.s_idx[tbase + s0 + c0 + jp];
          break;
        }
      }
      const uint32_t k = (uint32_t)key;
      const int kl = ((int)k - base) & (kWave - 1);
      PRT(9)
      PRC(5, ballot(lane == kl && (int)k != cj) ? 1 : 0);

      // 3) node k (ComputeBrokerApp3.cc:269-320): FIFO single server, record cached in its lane
      cache_node(k, kl);
      const UDiv div_k{readlane_u32(c_dv.m, kl), readlane_u32(c_dv.sh, kl)};
      const int64_t dl_k = readlane_i64(c_dl, kl), ul_k = readlane_i64(c_ul, kl);
      const int32_t tl = (int32_t)readlane_u32((uint32_t)ch.tl, kl);
      const int32_t npend0 = (int32_t)readlane_u32((uint32_t)ch.npend, kl);
      const int64_t tl_done = readlane_i64(ch.tl_done, kl);
      const uint64_t tl_C = (uint64_t)readlane_i64((int64_t)ch.tl_C, kl);
      const uint32_t tl_S = readlane_u32(ch.tl_S, kl);
      const int64_t base_done = tl >= 0 ? tl_done : INT64_MIN;
      if (!resume) {
        // k's own next advert changes its key; when k is idle the run's first task becomes its
        // head and that task's advert ends the run
        int64_t kb;
        if (npend0 > 0) {
          kb = readlane_i64(ch.hd_done, kl) + ul_k;
        } else {
          const uint32_t S0 = udiv(readlane_u32((uint32_t)cr, jp), div_k);
          const int64_t a0 = t + dl_k;  // (<= 2^62)
          const int64_t st0 = a0 > base_done ? a0 : base_done;
          kb = kNever;  // (past the tick range the run is refused below anyway)
          if (S0 < kRegSCap && st0 <= kMaxTick) kb = st0 + ticks_of(S0) + ul_k;  // (< 2^61 + 2^62 + 2^61)
        }
        if (jp + 1 < cnt && readlane_i64(ca, jp + 1) > kb) {
          // the next publish comes after k's advert: a run of one, whatever the other nodes'
          // adverts (any horizon is at least t: every advert before t has been applied)
          E = t;
        } else {
          // 4) run horizon (replay.hip's horizon_all_in, per pending node of the lane): an advert
          //    of j takes the decision from k = (busy_b, k) only with a busy value v <= thr_j =
          //    busy_b - (j > k) (BrokerBaseApp3.cc:273, ties -> the lower index), and j's adverts
          //    from its next one (at nxt_j, carrying v1 = offset) on fall by at most the seconds
          //    elapsed, so none comes before max(nxt_j, w_j - thr_j s); thr_j < 0: never
          const uint32_t busy_b = (uint32_t)(key >> 32), kk = (uint32_t)key;
          int64_t e_lane = kNever;
          for (uint32_t m = act; m; m &= m - 1u) {
            const int s = __builtin_ctz(m);
            const uint32_t j = (uint32_t)(base + s * kWave + lane);
            const int64_t thr = (int64_t)busy_b - (j > kk ? 1 : 0);
            if (j == kk || thr < 0) continue;  // (k's own advert bounds the run below)
            const int64_t x = vnxt[s * kWave];
            const uint32_t off = vwoff[s * kWave];
            const int64_t bnd = (uint64_t)thr >= off ? x : x + ticks_of(off - (uint32_t)thr);
            e_lane = bnd < e_lane ? bnd : e_lane;
          }
          E = (int64_t)wave_min_u64((uint64_t)e_lane);
          E = kb < E ? kb : E;
        }
      }
      // the run: publishes jp .. jq-1 of the segment (contiguous lanes: nondecreasing ticks)
      const uint64_t run_mask = ballot((lane >= jp && live && ca <= E) || lane == jp);
      const int jq = jp + __popcll(run_mask >> jp);
      const int Lr = jq - jp;
      const bool in_run = lane >= jp && lane < jq;
      const bool one = Lr == 1;  // a single publish needs no wave scans
      uint32_t S = 0u;
      int64_t a = 0;
      if (in_run) {
        S = udiv((uint32_t)cr, div_k);  // double tskTime = requiredMIPS / MIPS (:276)
        a = ca + dl_k;
      }
      // FIFO recurrence over the run: done_m = max(base, max_{i<=m} (a_i - P_{i-1})) + P_m
      const uint32_t Cs = one ? S : wave_scan_add_u32(in_run ? min(S, kRegSCap) : 0u);  // (< 64 * 2^22)
      // a service prefix of 2^22 s or more, or an arrival past 2^61 ticks, puts the run past the
      // tick range (the wide kernel's kPastRange): the sequential kernel decides the replication
      if (ballot(in_run && (Cs >= kRegSCap || a > kMaxTick))) {
        err = kRegionSeq;
        esc_hit = 0;
        break;
      }
      int64_t X = in_run ? a - ticks_of(Cs - S) : INT64_MIN;
      if (!one) X = wave_scan_max_i64(X);
      const int64_t dmax = base_done > X ? base_done : X;
      const int64_t start = dmax + ticks_of(Cs - S);
      const int64_t done = dmax + ticks_of(Cs);
      if (ballot(in_run && done > kMaxTick)) {
        err = kRegionSeq;
        esc_hit = 0;
        break;
      }
      int64_t prev_done = base_done;
      uint32_t prev_S = tl_S;
      if (!one) {
        const int64_t dn_up = dpp_or_i64<kDppWaveShr1>(0, done);
        const uint32_t S_up = dpp_or_u32<kDppWaveShr1>(0u, S);
        if (lane != jp) {
          prev_done = dn_up;
          prev_S = S_up;
        }
      }
      uint32_t status = 0u;
      if (in_run) {
        if (prev_done < a) status = 5u;       // idle: "task assigned" (:282-301)
        else if (prev_done > a) status = 4u;  // busy: "task queued" (:304-313)
        else status = dl_k < (int64_t)min(prev_S, kRegSCap) * kTicksPerSecond ? 5u : 4u;  // same-tick completion
        const int i = s0 + c0 + lane;  // the task's sorted position: chained in order on node k
        e[i] = WideEntry{a, done, tl_C + Cs, S, lane == jp ? tl : i - 1, lane + 1 < jq ? i + 1 : -1, 0};
        q_on = true;
        q_k = k;
        q_status = status;
        q_start = start;
        q_done = done;
      }
      // 5) node k's record after the run (owner lane)
      const int lz = jq - 1;
      const int64_t a_z = readlane_i64(a, lz), done_z = readlane_i64(done, lz);
      const uint32_t Cs_z = readlane_u32(Cs, lz), S_z = readlane_u32(S, lz);
      const int64_t done_f = readlane_i64(done, jp);
      const uint32_t S_f = readlane_u32(S, jp);
      if (lane == kl) {
        WideNode h = ch;
        const int i0 = s0 + c0 + jp, iz = s0 + c0 + lz;
        const int sk = ((int)k - base) / kWave;
        if (h.npend == 0) {  // the run's first task is the node's head: its advert is the node's next one
          h.hd = i0;
          h.hd_done = done_f;
          h.hd_C = tl_C + S_f;
          h.hd_S = S_f;
          const int64_t x = done_f + ul_k;
          vnxt[sk * kWave] = x;
          act |= 1u << sk;
          if (x < mn) {
            mn = x;
            ms = sk;
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
        h.tl_C = tl_C + Cs_z;
        h.tl_S = S_z;
        h.npend += Lr;
        ch = h;
        max_pend = max(max_pend, (uint32_t)h.npend);
        vwoff[sk * kWave] = (uint16_t)w_offset(h, dl_k);  // k's horizon offset
      }
      n_done += Lr;
      PRC(6, Lr);
      PRT(10)
      if (jq == cnt) {  // the chunk is used up and E still bounds the decision
        carry = true;
        E_carry = E;
      }
      jp = jq;
    }
    // the chunk's outputs (pushed lanes, coalesced, region-sorted order)
    if (q_on) {
      const size_t o = tbase + (size_t)(s0 + c0 + lane);
      W.o_node[o] = (int32_t)q_k;
      W.o_status[o] = (uint8_t)q_status;
      W.o_start[o] = q_start;
      W.o_done[o] = q_done;
    }
  }
  if (cj >= 0) {
    nd[cj] = ch;
    write_tail(cj, ch);
  }
#ifdef FOGNET_REGION_PROF
  pr[11] = clock64() - pt0;
  if (lane == 0 && (blockIdx.x < 3 || blockIdx.x % 997 == 7))
    printf("RPROF blk %d iters %lu resumed %lu advrounds %lu adverts %lu advhit %lu kmiss %lu pubs %lu cyc_pre %lu "
           "cyc_adv %lu cyc_dec %lu cyc_run %lu cyc_tot %lu\n",
           (int)blockIdx.x, pr[0], pr[1], pr[2], pr[3], pr[4], pr[5], pr[6], pr[7], pr[8], pr[9], pr[10], pr[11]);
#endif
  const uint32_t mp = ~wave_min_u32(~max_pend);
  if (lane == 0) {
    if (PASS == 1 && esc_hit >= 0) atomicMin(W.esc + r, esc_hit);
    W.rec[rb] = RegionRec{n_done, (int32_t)mp, (int32_t)err, 0};
  }
}

// Per replication (256 threads): the regions' records merged, the node tails'
// busy seconds and last completion (FIFO: the tail's cumulative service and
// completion), then the statistics pass in trace order -- each task's outputs
// gathered from its sorted position, written to the caller's arrays and
// accumulated (the fused epilogue's arithmetic) -- by waves 1-3 while wave 0
// sums the a11 energy in node order (replay_wide.hip's order): the energy's
// serial chain needs only the last completion.  A replication some region could
// not finish goes to the hand-over list instead.
constexpr int kFinThreads = 256;  // wave 0: the energy chain; waves 1-3: the statistics pass

__global__ __launch_bounds__(kFinThreads) void region_finish_kernel(ReplayArgs A, RegionWs W) {
  const int r = blockIdx.x;
  const int tid = threadIdx.x;
  const int B = W.B, N = A.N;
  constexpr int kFinWaves = kFinThreads / kWave;
  constexpr int kStatThreads = kFinThreads - kWave;  // waves 1..3
  // (per-wave partial records: 4 x 152 B of LDS)
  __shared__ Acc s_acc[kFinWaves];
  __shared__ int64_t s_abt[kFinThreads];
  __shared__ int32_t s_abk[kFinThreads];
  __shared__ uint32_t s_hist[FOGNET_HIST_METRICS * FOGNET_HIST_BINS];
  __shared__ int s_ok, s_done, s_mp;
  __shared__ double s_energy;
  __shared__ double s_ebuf[kWave];  // the energy chain's terms, one chunk at a time
  __shared__ uint64_t s_busy;
  __shared__ int64_t s_last;
  if (tid < kWave) {  // the regions' records, one per lane (B <= 64: N <= 65,536)
    RegionRec x{0, 0, FOGNET_OK, 0};
    if (tid < B) x = W.rec[(size_t)r * B + tid];
    const bool ok = ballot(x.status != FOGNET_OK) == 0ull;
    const int done = (int)wave_sum_u32((uint32_t)x.n_done);
    const int mp = (int)~wave_min_u32(~(uint32_t)x.max_pend);
    if (tid == 0) {
      s_ok = ok;
      s_done = done;
      s_mp = mp;
    }
  }
  __syncthreads();
  // resume (second pass run): the second pass replayed r up to its first escalated publish esc;
  // the publishes before it are finished here, and the sequential kernel continues from esc
  const int32_t esc = W.esc[r];
  const bool part = W.pass == 2 && A.wide_list && esc > 0 && esc < A.T;
  if (!s_ok || (part && s_done != esc)) {  // the sequential replay overwrites the record
    if (tid == 0) {
      // (FOGNET_HIER_REGIONS=only: no hand-over list, the replication stays unreplayed)
      A.out_stats[r].status = A.wide_list ? kRegionSeq : FOGNET_ERR_UNSUPPORTED;
      if (W.pass == 2) W.esc[r] = 0;  // from the start
      if (A.wide_list) A.wide_list[atomicAdd(A.wide_count, 1)] = r;
    }
    return;
  }
  const int n = s_done;  // == T, or esc (part)
  fognet_rep_stats* const S = A.out_stats + r;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)A.T;
  for (int h = tid; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kFinThreads) s_hist[h] = 0u;
  s_abt[tid] = INT64_MAX;
  s_abk[tid] = INT32_MAX;
  // busy seconds and the last completion from the node tails (the region pass's compact copy,
  // 16 B per node; four in flight per thread)
  const int64_t* const tails = W.tails + 2 * (size_t)r * (size_t)N;
  Acc a = acc_identity();
  for (int j0 = tid; j0 < N; j0 += 4 * kFinThreads) {
    int64_t td[4], tc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * kFinThreads;
      td[u] = j < N ? tails[2 * (size_t)j] : INT64_MIN;
      tc[u] = j < N ? tails[2 * (size_t)j + 1] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a.busy += (uint64_t)tc[u];
      a.last = max(a.last, td[u]);
    }
  }
  a = wave_merge(a);
  if ((tid & (kWave - 1)) == 0) s_acc[tid / kWave] = a;
  __syncthreads();
  if (tid == 0) {
    uint64_t busy = 0u;
    int64_t last = INT64_MIN;
#pragma unroll 1
    for (int w = 0; w < kFinWaves; ++w) {
      busy += s_acc[w].busy;
      last = max(last, s_acc[w].last);
    }
    s_busy = busy;
    s_last = last;
  }
  __syncthreads();  // (s_acc is reused below)
  if (tid < kWave) {
    // a11 energy (fognet_hip.h): E_j = P_busy_j * B_j + P_idle_j * ((H - B_j 1e12) / 1e12), summed in
    // node order (64 nodes at a time, then lane by lane) while waves 1-3 run the statistics pass
    // (part: the sequential kernel sums it at the end)
#ifndef FOGNET_FIN_NOENERGY
    if (A.p_busy && !part) {  // (an unused node's record has tl_C = 0)
#else
    if (false) {  // timing probe only
#endif
      const int64_t H = n > 0 ? s_last : 0;
      const double sum = energy_sum_wave(reinterpret_cast<const uint64_t*>(tails) + 1, 2, A.p_busy + nbase,
                                         A.p_idle + nbase, N, H,
                                         A.out_energy ? A.out_energy + (size_t)r * (size_t)N : nullptr, tid, s_ebuf);
      if (tid == 0) s_energy = sum;
    }
  } else {
    // tasks i = i0, i0 + 192, ... in trace order: position p = inv[i]; the outputs gathered from p,
    // written to task i, and accumulated (stats_accumulate's arithmetic, task index i)
    constexpr int U = 4;  // (two dependent loads per task: keep 8 in flight)
    const int i0 = tid - kWave;
    const bool hist = A.hist != nullptr;
    Acc b = acc_identity();
#ifdef FOGNET_FIN_NOSTATS
    for (int ib = n; ib < n; ib += kStatThreads * U) {  // timing probe only
#else
    for (int ib = i0; ib < n; ib += kStatThreads * U) {
#endif
      int64_t t[U], st0[U], dn[U];
      int32_t kk[U], pp[U];
      uint32_t stt[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = ib + u * kStatThreads;
        const size_t o = tbase + (size_t)(i < n ? i : ib);  // past the end: reload task ib (in bounds, unused)
        t[u] = A.arrive[o];
        pp[u] = W.inv[o];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const size_t p = tbase + (size_t)pp[u];
        kk[u] = W.o_node[p];
        stt[u] = W.o_status[p];
        st0[u] = W.o_start[p];
        dn[u] = W.o_done[p];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = ib + u * kStatThreads;
        if (i < n) {
          const size_t o = tbase + (size_t)i;
          A.out_node[o] = kk[u];
          A.out_status[o] = (uint8_t)stt[u];
          A.out_start[o] = st0[u];
          A.out_done[o] = dn[u];
          const int64_t resp = dn[u] - t[u];
          add_moment(b.rs_lo, b.rs_hi, b.rq_lo, b.rq_hi, (uint64_t)resp);
          b.rmin = min(b.rmin, resp);
          b.rmax = max(b.rmax, resp);
          if (hist) atomicAdd(&s_hist[FOGNET_HIST_BINS + hist_bin(resp)], 1u);
          if (stt[u] == 4u) {  // queueTime emission (ComputeBrokerApp3.cc:238), enqueued at its arrival
            b.n4 += 1u;
            if (!acc_qtime(b.qs_lo, b.qs_hi, b.qq_lo, b.qq_hi, b.qq_top, b.qmin, b.qmax, b.nqt, b.nqo, st0[u],
                           t[u] + A.dl[nbase + kk[u]], hist ? s_hist : nullptr))
              abort_min(s_abt[tid], s_abk[tid], st0[u], i);
          } else {
            b.n5 += 1u;
          }
        }
      }
    }
    b = wave_merge(b);
    const AbortPt ab_w = wave_min_abort(AbortPt{s_abt[tid], s_abk[tid]});  // (each thread's own slot)
    if ((tid & (kWave - 1)) == 0) {
      s_acc[tid / kWave] = b;
      s_abt[tid] = ab_w.tick;
      s_abk[tid] = ab_w.task;
    }
  }
  __syncthreads();
  if (tid == 0) {
    Acc t = s_acc[1];
    AbortPt ab = AbortPt{s_abt[kWave], s_abk[kWave]};
#pragma unroll 1
    for (int w = 2; w < kFinWaves; ++w) {
      acc_merge(t, s_acc[w]);
      abort_min(ab.tick, ab.task, s_abt[w * kWave], s_abk[w * kWave]);
    }
    t.busy = s_busy;  // (the node tails': the statistics pass adds none)
    t.last = s_last;
    if (part) {  // the publishes before esc: the record the sequential kernel starts from
      static_assert(sizeof(Acc) + sizeof(AbortPt) <= kRegionResumeBytes, "resume record");
      unsigned char* const pr = W.pacc + (size_t)r * kRegionResumeBytes;
      *reinterpret_cast<Acc*>(pr) = t;
      *reinterpret_cast<AbortPt*>(pr + sizeof(Acc)) = ab;
      S->status = kRegionSeq;
      A.wide_list[atomicAdd(A.wide_count, 1)] = r;
    } else {
      S->n_tasks = n;
      S->max_pending = s_mp;
      S->status = FOGNET_OK;
      S->events = 2 * (int64_t)N + 4 * (int64_t)n;  // initial adverts + publish, arrival, release, advert per task
      write_rep_stats(S, t, ab, A.ref_abort);
      if (A.p_busy) S->energy_j = s_energy;
    }
  }
  if (A.hist) {
    for (int h = tid; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kFinThreads)
      if (s_hist[h]) atomicAdd((unsigned long long*)&A.hist[h], (unsigned long long)s_hist[h]);
  }
}

}  // namespace

hipError_t launch_replay_region(const ReplayArgs& a, const RegionWs& w, bool resume, hipStream_t s) {
  RegionWs w1 = w;
  w1.pass = 1;
  hipLaunchKernelGGL(region_sort_kernel, dim3(a.R), dim3(kSortThreads), 0, s, a, w1);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(region_order_kernel, dim3(1), dim3(kOrderThreads), 0, s, (int32_t)(a.R * w.B), w1);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(replay_region_kernel<1>, dim3((unsigned)a.R * (unsigned)w.B), dim3(kWave), 0, s, a, w1);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  RegionWs w2 = w;
  w2.pass = resume ? 2 : 1;  // (the finish kernel: whether the second pass ran)
  if (resume) {  // the escalated replications again, each region exactly up to the first escalation
    hipLaunchKernelGGL(replay_region_kernel<2>, dim3((unsigned)a.R * (unsigned)w.B), dim3(kWave), 0, s, a, w2);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(region_finish_kernel, dim3(a.R), dim3(kFinThreads), 0, s, a, w2);
  return hipGetLastError();
}

}  // namespace fognet
