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
// replayed by its own wavefront over the region's publishes only: B waves per
// replication instead of one, each walking a tenth of the chain.  The same
// closed form as replay_wide.hip: node j of region b (local
// index l = j - 1024 b) lives on lane l % 64, slot l / 64, with its view
// (next advert tick, advertised busy) in this lane's registers (16 slots), its
// record (WideNode) and its tasks' chain (WideEntry) in HBM.
//
// A replication in which any region meets an escalation (or anything else this
// kernel does not model: a saturated busy time, a service time past 2^22 s, an
// invalid input) is replayed again from the start by the sequential wide
// kernel (the hand-over list, like the register kernel's), which defines every
// result of such a replication; nothing of this pass survives for it.  For the
// others region_finish_kernel merges the regions' records and runs the
// statistics pass over the per-task outputs (the same Acc record, histogram and
// a11 energy as the wide kernel's inline statistics).
#include "replay_common.h"

namespace fognet {

namespace {

constexpr int kRegionSlots = FOGNET_HIER_REGION_NODES / kWave;  // 16 view slots per lane
static_assert(kRegionSlots == kWideGroupSlots, "a region is one wide-kernel group row");
constexpr uint32_t kRegBusySat = 0xFFFFFFFFu;
constexpr uint32_t kRegSCap = 1u << 22;  // the wide kernel's kWideSCap: past it the sequential kernel decides

// Internal per-(replication, region) status: replay the replication sequentially
// (fognet_hip.h never returns it; tests see it under FOGNET_HIER_REGIONS=only).
constexpr int32_t kRegionSeq = 0x53455121;
constexpr int kQuitEvery = 4;  // chunks between polls of the replication's quit flag

// 4 waves per SIMD: 8 KiB of LDS each (the view's ticks), <= 128 VGPRs.
__global__ __launch_bounds__(64, 4) void replay_region_kernel(ReplayArgs A, RegionWs W) {
  const int B = W.B;
  const int r = blockIdx.x / B, b = blockIdx.x - (blockIdx.x / B) * B;
  const int rb = r * B + b;  // (r, b)'s region record and busy view
  const int lane = threadIdx.x;
  const int T = A.T, N = A.N;
  const int base = b * FOGNET_HIER_REGION_NODES;
  const int nb = min(FOGNET_HIER_REGION_NODES, N - base);  // nodes of this region (>= 1)
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  WideEntry* const e = W.e + tbase;
  WideNode* const nd = W.nd + (size_t)r * (size_t)N;
  const int64_t arrive0 = T > 0 ? A.arrive[tbase] : kNever;

  // ---- this lane's nodes (local l = s * 64 + lane) and their view ([slot][lane]: each lane
  // touches only its own column): next advert ticks in LDS (conflict-free); advertised busy
  // times in HBM (RegionWs::vb; read back only by a key rescan of a lane without a zero-busy
  // slot), so the LDS of a wavefront is 8 KiB: 20 fit per CU, and 4 per SIMD by VGPRs
  __shared__ int64_t s_nxt[kRegionSlots * kWave];
  int64_t* const vnxt = s_nxt + lane;  // vnxt[s * kWave]: slot s of this lane
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
    vbusy[s * kWave] = l < nb ? 0u : kRegBusySat;  // (past the region: never the minimum)
    nzb |= l < nb ? 0u : 1u << s;
    if (l < nb) {
      const int j = base + l;
      const int32_t m = A.mips[nbase + j];
      const int64_t d = A.dl[nbase + j], u = A.ul[nbase + j], ia = A.init[nbase + j];
      bad |= (m <= 0) | (d < 0) | (u < 0) | (d > kMaxTick) | (u > kMaxTick) | (ia < u) | (ia >= arrive0);
      nd[j] = WideNode{-1, -1, 0, -1, 0, 0u, 0, 0, 0u, 0u, 0u};
    }
  }
  // the lane's earliest advert (slot ms) and smallest view key (busy << 32 | j)
  int64_t mn = kNever;
  int ms = 0;
  uint64_t mk = lane < nb ? (uint64_t)(uint32_t)(base + lane) : ~0ull;
  // after slot sl's view tick became xs: the earliest over the pending slots (ties: the
  // smallest slot)
  auto rescan_nxt = [&](int sl, int64_t xs) {
    mn = xs;
    ms = sl;
    for (uint32_t m = act & ~(1u << sl); m; m &= m - 1u) {
      const int s = __builtin_ctz(m);
      const int64_t x = vnxt[s * kWave];
      if (x < mn || (x == mn && s < ms)) {
        mn = x;
        ms = s;
      }
    }
  };
  // (partially unrolled: a full unroll issues all 16 LDS loads at once and holds 32 VGPRs)
  auto rescan_key = [&]() {
    const uint32_t z = ~nzb & ((1u << kRegionSlots) - 1u);
    if (z) {  // a zero-busy slot: the smallest one holds the smallest key
      mk = (uint32_t)(base + __builtin_ctz(z) * kWave + lane);
      return;
    }
    mk = ~0ull;
#pragma unroll 1
    for (int s0 = 0; s0 < kRegionSlots; s0 += 8) {  // (8 loads in flight: few registers)
      uint32_t bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) bv[u] = vbusy[(s0 + u) * kWave];
      sync_vm();  // (in this arm: see sync_vm)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint64_t key = ((uint64_t)bv[u] << 32) | (uint32_t)(base + (s0 + u) * kWave + lane);
        mk = key < mk ? key : mk;
      }
    }
  };

  uint32_t err = ballot(bad) ? (uint32_t)kRegionSeq : (uint32_t)FOGNET_OK;
  uint32_t max_pend = 0u;
  int n_done = 0;
  int64_t prev_t = INT64_MIN;
  // the node this lane pushed to last (the stale view keeps choosing it): its
  // record and parameters in registers, written back when the lane pushes to
  // another node and at the end (replay_wide.hip's cache)
  int cj = -1;
  WideNode ch{};
  UDiv c_dv{1u, 0u};
  int64_t c_dl = 0, c_ul = 0;
  auto cache_node = [&](uint32_t kk, int kl) {
    if (lane == kl && (int)kk != cj) {
      if (cj >= 0) nd[cj] = ch;


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
#ifdef FOGNET_REGION_PROF
  uint64_t pr[16] = {};
  uint64_t pt0 = clock64(), pt = 0;
#define PRC(i, v) pr[i] += (v)
#define PRT(i) { const uint64_t _n = clock64(); pr[i] += _n - pt; pt = _n; }
#else
#define PRC(i, v)
#define PRT(i)
#endif

  for (int c0 = 0; c0 < T && err == FOGNET_OK; c0 += kWave) {
    // another region of r handed it back: the sequential kernel replays r from the start
    if ((c0 & (kQuitEvery * kWave - 1)) == 0 && c0 > 0 &&
        __hip_atomic_load(W.quit + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
      err = kRegionSeq;
      break;
    }
    const int cnt = min(kWave, T - c0);
    const bool live = lane < cnt;
    const int64_t ca = live ? A.arrive[tbase + c0 + lane] : kNever;
    const int32_t cr = live ? A.req[tbase + c0 + lane] : 0;
    const int32_t cg = live ? A.region[tbase + c0 + lane] : 0;
    // trace preconditions (the sequential kernel reports them)
    const int64_t prv = dpp_or_i64<kDppWaveShr1>(prev_t, ca);  // lane 0 gets prev_t
    if (ballot(live && (ca < prv || cr < 0 || ca > kMaxTick || cg < 0 || cg >= B))) {
      err = kRegionSeq;
      break;
    }
    prev_t = readlane_i64(ca, cnt - 1);
    // this chunk's publishes of region b; each member lane keeps its task's outputs until the chunk ends
    uint64_t mem = ballot(live && cg == b);
#ifdef FOGNET_REGION_PROF
    pt = clock64();
#endif
    bool q_on = false;
    uint32_t q_k = 0u, q_status = 0u;
    int64_t q_start = 0, q_done = 0;
    while (mem) {
      const int jp = (int)__builtin_ctzll(mem);
      mem &= mem - 1ull;
      const int64_t t = readlane_i64(ca, jp);

      // 1) completion adverts that reached the broker strictly before t, lane-parallel
      bool lbroken = false;
      if (ballot(mn < t)) view_changed = true;
      PRC(0, 1);
      while (ballot(mn < t)) {
        PRC(1, 1);
        PRC(2, __builtin_popcountll(ballot(mn < t)));
        PRC(3, __builtin_popcountll(ballot(mn < t && base + ms * kWave + lane == cj)));
        PRC(4, __builtin_popcountll(ballot(mn < t && base + ms * kWave + lane == cj && ch.npend >= 2)));
        if (mn < t) {
          const int sl = ms;
          const int j = base + sl * kWave + lane;
          const bool hit = j == cj;
          int64_t nxt_j;
          uint32_t busy_j;
          bool broken = false;
          // the cached record is updated in place (no copy of it through a merged value)
          if (hit) {
            (void)apply_wide_advert(ch, e, c_dl, c_ul, 0, nxt_j, busy_j, broken);
            while (nxt_j < t && !broken) (void)apply_wide_advert(ch, e, c_dl, c_ul, 0, nxt_j, busy_j, broken);
          } else {  // (waited for here, not where the arms meet: sync_vm)
            WideNode h = nd[j];
            const int64_t dl_j = A.dl[nbase + j], ul_j = A.ul[nbase + j];
            sync_vm();
            (void)apply_wide_advert(h, e, dl_j, ul_j, 0, nxt_j, busy_j, broken);
            while (nxt_j < t && !broken) (void)apply_wide_advert(h, e, dl_j, ul_j, 0, nxt_j, busy_j, broken);
            nd[j] = h;
          }
          lbroken |= broken;
          vnxt[sl * kWave] = nxt_j;
          vbusy[sl * kWave] = busy_j;
          act = nxt_j != kNever ? act | (1u << sl) : act & ~(1u << sl);
          nzb = busy_j != 0u ? nzb | (1u << sl) : nzb & ~(1u << sl);
          rescan_nxt(sl, nxt_j);
          // the key: only j's changed; a rescan only when j held the minimum and grew
          const uint64_t nk = ((uint64_t)busy_j << 32) | (uint32_t)j;
          PRC(6, __builtin_popcountll(ballot((uint32_t)mk == (uint32_t)j && nk > mk)));
          if ((uint32_t)mk == (uint32_t)j && nk > mk) rescan_key();
          else mk = nk < mk ? nk : mk;
        }
      }
      if (ballot(lbroken)) {
        err = FOGNET_ERR_INTERNAL;
        break;
      }
      PRT(8)
      // 2) the regional broker's decision; above the threshold it would escalate
      PRC(7, view_changed ? 1 : 0);
      if (view_changed) {
        key = wave_min_u64(mk);
        view_changed = false;
      }
      if ((key >> 32) > (uint64_t)A.hier_thr || (key >> 32) >= kRegBusySat) {
        err = kRegionSeq;
        break;
      }
      const uint32_t k = (uint32_t)key;
      const int kl = ((int)k - base) & (kWave - 1);

      // 3) the task reaches node k (ComputeBrokerApp3.cc:269-320): FIFO single server
      PRC(5, ballot(lane == kl && (int)k != cj) ? 1 : 0);
      PRC(12, (k - base) / kWave);
      PRT(9)
      cache_node(k, kl);
      const UDiv div_k{readlane_u32(c_dv.m, kl), readlane_u32(c_dv.sh, kl)};
      const int64_t dl_k = readlane_i64(c_dl, kl), ul_k = readlane_i64(c_ul, kl);
      const int32_t tl = (int32_t)readlane_u32((uint32_t)ch.tl, kl);
      const int64_t tl_done = readlane_i64(ch.tl_done, kl);
      const uint64_t tl_C = (uint64_t)readlane_i64((int64_t)ch.tl_C, kl);
      const uint32_t tl_S = readlane_u32(ch.tl_S, kl);
      const uint32_t S = udiv(readlane_u32((uint32_t)cr, jp), div_k);  // double tskTime = requiredMIPS / MIPS (:276)
      const int64_t a = t + dl_k;
      const int64_t base_done = tl >= 0 ? tl_done : INT64_MIN;
      const int64_t start = a > base_done ? a : base_done;
      // (a <= 2^62 and S < 2^22: no int64 overflow below)
      const int64_t done = S < kRegSCap ? start + ticks_of(S) : kNever;
      if (a > kMaxTick || done > kMaxTick) {  // past the tick range: the sequential kernel refuses it
        err = kRegionSeq;
        break;
      }
      uint32_t status;
      if (base_done < a) status = 5u;       // idle: "task assigned" (:282-301)
      else if (base_done > a) status = 4u;  // busy: "task queued" (:304-313)
      else status = dl_k < (int64_t)min(tl_S, kRegSCap) * kTicksPerSecond ? 5u : 4u;  // same-tick completion
      const int i = c0 + jp;
      const uint64_t C = tl_C + S;
      if (lane == kl) {
        e[i] = WideEntry{a, done, C, S, tl, -1, 0};
        WideNode h = ch;
        // (no three-way branch on npend: that shape, with a store in the middle arm, was
        // miscompiled on gfx950 -- DESIGN.md §3.6 "The hd_next miscompile"; hd_next is set
        // after the two-way branch instead)
        if (h.npend == 0) {  // the task is the node's head: its advert is the node's next one
          h.hd = i;
          h.hd_done = done;
          h.hd_C = C;
          h.hd_S = S;
          const int sk = ((int)k - base) / kWave;
          const int64_t x = done + ul_k;
          vnxt[sk * kWave] = x;
          act |= 1u << sk;
          if (x < mn) {
            mn = x;
            ms = sk;
          }
        } else if (h.npend >= 2) {
          e[h.tl].next = i;
        }
        if (h.npend == 1) h.hd_next = i;  // the tail is the head
        h.tl = i;
        h.tl_a = a;
        h.tl_done = done;
        h.tl_C = C;
        h.tl_S = S;
        h.npend += 1;
        ch = h;
        max_pend = max(max_pend, (uint32_t)h.npend);
      }
      if (lane == jp) {
        q_on = true;
        q_k = k;
        q_status = status;
        q_start = start;
        q_done = done;
      }
      n_done += 1;
      PRT(10)
    }
    // the chunk's outputs (member lanes, coalesced)
    if (q_on) {
      const size_t o = tbase + (size_t)(c0 + lane);
      A.out_node[o] = (int32_t)q_k;
      A.out_status[o] = (uint8_t)q_status;
      A.out_start[o] = q_start;
      A.out_done[o] = q_done;
    }
  }
  if (cj >= 0) nd[cj] = ch;
#ifdef FOGNET_REGION_PROF
  pr[11] = clock64() - pt0;
  if (lane == 0 && (blockIdx.x < 3 || blockIdx.x % 1000 == 7))
    printf("RPROF blk %d pubs %lu rounds %lu advl %lu hit %lu hit_e %lu cmiss %lu krescan %lu dec %lu cyc_adv %lu cyc_dec %lu cyc_push %lu cyc_tot %lu slotsum %lu\n",
           (int)blockIdx.x, pr[0], pr[1], pr[2], pr[3], pr[4], pr[5], pr[6], pr[7], pr[8], pr[9], pr[10], pr[11], pr[12]);
#endif
  const uint32_t mp = ~wave_min_u32(~max_pend);
  if (lane == 0) {
    if (err != FOGNET_OK) __hip_atomic_store(W.quit + r, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    W.rec[rb] = RegionRec{n_done, (int32_t)mp, (int32_t)err, 0};
  }
}

// Per replication (256 threads): the regions' records merged, the node tails'
// busy seconds and last completion (FIFO: the tail's cumulative service and
// completion), then the statistics pass over the outputs (stats_accumulate, the
// fused epilogue's code) by waves 1-3 while wave 0 sums the a11 energy in node
// order (replay_wide.hip's order): the energy's serial chain needs only the last
// completion.  A replication some region could not finish goes to the hand-over
// list instead.
constexpr int kFinThreads = 256;

__global__ __launch_bounds__(kFinThreads) void region_finish_kernel(ReplayArgs A, RegionWs W) {
  const int r = blockIdx.x;
  const int tid = threadIdx.x;
  const int B = W.B, N = A.N;
  constexpr int kFinWaves = kFinThreads / kWave;
  constexpr int kStatThreads = kFinThreads - kWave;  // waves 1..3
  // (per-wave partial records: 4 x 152 B of LDS, so many blocks fit per CU)
  __shared__ Acc s_acc[kFinWaves];
  __shared__ int64_t s_abt[kFinThreads];
  __shared__ int32_t s_abk[kFinThreads];
  __shared__ uint32_t s_hist[FOGNET_HIST_METRICS * FOGNET_HIST_BINS];
  __shared__ int s_ok, s_done, s_mp;
  __shared__ double s_energy;
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
  if (!s_ok) {  // the sequential replay overwrites the record
    if (tid == 0) {
      // (FOGNET_HIER_REGIONS=only: no hand-over list, the replication stays unreplayed)
      A.out_stats[r].status = A.wide_list ? kRegionSeq : FOGNET_ERR_UNSUPPORTED;
      if (A.wide_list) A.wide_list[atomicAdd(A.wide_count, 1)] = r;
    }
    return;
  }
  const int n = s_done;  // == T
  fognet_rep_stats* const S = A.out_stats + r;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)A.T;
  const WideNode* const nd = W.nd + (size_t)r * (size_t)N;
  for (int h = tid; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kFinThreads) s_hist[h] = 0u;
  s_abt[tid] = INT64_MAX;
  s_abk[tid] = INT32_MAX;
  // busy seconds and the last completion from the node tails (2 records in flight per thread)
  Acc a = acc_identity();
  for (int j0 = tid; j0 < N; j0 += 2 * kFinThreads) {
    WideNode x[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = j0 + u * kFinThreads;
      x[u] = j < N ? nd[j] : WideNode{-1, -1, 0, -1, 0, 0u, 0, 0, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (x[u].tl >= 0) {
        a.busy += x[u].tl_C;
        a.last = max(a.last, x[u].tl_done);
      }
    }
  }
  a = wave_merge(a);
  if ((tid & (kWave - 1)) == 0) s_acc[tid / kWave] = a;
  __syncthreads();
  if (tid == 0) {
    uint64_t busy = 0u;
    int64_t last = INT64_MIN;
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
    if (A.p_busy) {  // (an unused node's record has tl_C = 0)
      const int64_t H = n > 0 ? s_last : 0;
      const double sum = energy_sum_wave(nd, A.p_busy + nbase, A.p_idle + nbase, N, H,
                                         A.out_energy ? A.out_energy + (size_t)r * (size_t)N : nullptr, tid);
      if (tid == 0) s_energy = sum;
    }
  } else {
    Acc b = acc_identity();
    stats_accumulate<2, false>(A, tbase, n, tid - kWave, kStatThreads, b, nullptr, s_hist,
                               [&](int k) { return A.dl[nbase + k]; }, s_abt + kWave, s_abk + kWave);
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
    for (int w = 2; w < kFinWaves; ++w) {
      acc_merge(t, s_acc[w]);
      abort_min(ab.tick, ab.task, s_abt[w * kWave], s_abk[w * kWave]);
    }
    t.busy = s_busy;  // (the node tails': the statistics pass adds none)
    t.last = s_last;
    S->n_tasks = n;
    S->max_pending = s_mp;
    S->status = FOGNET_OK;
    S->events = 2 * (int64_t)N + 4 * (int64_t)n;  // initial adverts + publish, arrival, release, advert per task
    write_rep_stats(S, t, ab, A.ref_abort);
    if (A.p_busy) S->energy_j = s_energy;
  }
  if (A.hist) {
    for (int h = tid; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kFinThreads)
      if (s_hist[h]) atomicAdd((unsigned long long*)&A.hist[h], (unsigned long long)s_hist[h]);
  }
}

}  // namespace

hipError_t launch_replay_region(const ReplayArgs& a, const RegionWs& w, hipStream_t s) {
  hipLaunchKernelGGL(replay_region_kernel, dim3((unsigned)a.R * (unsigned)w.B), dim3(kWave), 0, s, a, w);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(region_finish_kernel, dim3(a.R), dim3(kFinThreads), 0, s, a, w);
  return hipGetLastError();
}

}  // namespace fognet
