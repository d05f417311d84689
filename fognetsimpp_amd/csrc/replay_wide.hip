// replay_wide.hip — batched trace replay for large fog-node sets on gfx950
// (BASELINE.json configs[4], C5: 10,000 fog nodes; here N <= 13,568).  Same
// reference semantics and the same closed form as replay.hip,
// restated for node sets that do not fit in registers:
//   decision   BrokerBaseApp3::sendPubAck(status=false)   BrokerBaseApp3.cc:265-304
//   arrival    ComputeBrokerApp3::processPacket (task)     ComputeBrokerApp3.cc:269-320
//   completion ComputeBrokerApp3::releaseResource          ComputeBrokerApp3.cc:224-256
//   advert     advertiseMIPS + broker view update          ComputeBrokerApp3.cc:205-222,
//                                                          BrokerBaseApp3.cc:123-130
//
// One wavefront replays one replication.  Node j belongs to lane j % 64 and
// only that lane reads or writes node j's state, so the loop needs no
// barriers:
//   LDS    s_nxt[N]   i64  tick at which the advert of node j's head completion
//                          reaches the broker (kNever: nothing pending)
//          s_busy[N]  u32  the broker's advertised busyTime of node j (seconds)
//   VGPRs  per lane: the minimum of s_nxt and of the view key (busy << 32 | j)
//          over the lane's nodes, rescanned from LDS after the lane applies an
//          advert
//   HBM    WideEntry [R][T]: per task its arrival, completion, cumulative
//          service and the links of its node's pending chain;
//          WideNode [R][N]: head, tail and pending count of each node.
// Publishes are decided one at a time in trace order: adverts that reached
// the broker strictly before the publish are applied first (lane-parallel:
// adverts of different nodes commute, those of one node come in completion
// order), the decision is a wave-wide u64 minimum of the lane minima (ties ->
// lowest index, the strict '<' of BrokerBaseApp3.cc:273), and the owner lane
// of the chosen node appends the task and accumulates its statistics (the
// same record replay.hip's fused epilogue writes).
#include "replay_common.h"

namespace fognet {

namespace {

constexpr uint32_t kWideMaxS = 0xFFFFu;  // service seconds < 2^16 (kMaxTick arithmetic)

// Lane-local rescan of the lane's nodes: earliest pending advert and smallest view key.
__device__ __forceinline__ void lane_scan(const int64_t* s_nxt, const uint32_t* s_busy, int N, int lane,
                                          int64_t& mn, int& mj, uint64_t& mk) {
  mn = kNever;
  mj = lane;
  mk = ~0ull;
  for (int j = lane; j < N; j += kWave) {
    const int64_t x = s_nxt[j];
    if (x < mn) {
      mn = x;
      mj = j;
    }
    const uint64_t key = ((uint64_t)s_busy[j] << 32) | (uint32_t)j;
    mk = key < mk ? key : mk;
  }
}

// The advert of node j's head completion reaches the broker (owner lane):
// the view takes busyTime after releaseResource (ComputeBrokerApp3.cc:232,
// :254) = the service of the tasks that reached j before that completion and
// are not done yet, a difference of cumulative sums; the head advances.
// Returns false when the advertised busy time does not fit 32 bits.
__device__ __forceinline__ bool apply_advert(int j, WideNode* nd, const WideEntry* e, int64_t dl, int64_t ul,
                                             int64_t* s_nxt, uint32_t* s_busy) {
  WideNode h = nd[j];
  const WideEntry hd = e[h.hd];
  uint64_t c_arrived = hd.C;            // only the completing task itself ...
  for (int32_t x = h.tl; x != h.hd;) {  // ... unless a newer one arrived first
    const WideEntry ex = e[x];
    if (arrives_before(ex.a, hd.done, dl, hd.S)) {
      c_arrived = ex.C;
      break;
    }
    x = ex.prev;
  }
  const uint64_t busy = c_arrived - hd.C;
  s_busy[j] = (uint32_t)busy;
  h.npend -= 1;
  if (h.npend == 0) {
    s_nxt[j] = kNever;
  } else {
    h.hd = hd.next;
    s_nxt[j] = e[hd.next].done + ul;  // FIFO: the next task started at max(arrival, this completion)
  }
  nd[j] = h;
  return busy < 0xFFFFFFFFull;
}

template <int POL>
__global__ __launch_bounds__(64) void replay_wide_kernel(ReplayArgs A, WideEntry* E, WideNode* ND) {
  constexpr bool kExt = POL == FOGNET_POLICY_EXT_LAT;
  extern __shared__ __align__(16) unsigned char w_lds[];
  const int r = blockIdx.x;
  const int lane = threadIdx.x;
  const int T = A.T, N = A.N;
  int64_t* const s_nxt = reinterpret_cast<int64_t*>(w_lds);
  uint32_t* const s_busy = reinterpret_cast<uint32_t*>(s_nxt + N);
  uint32_t* const s_hist = s_busy + N;  // [FOGNET_HIST_METRICS][FOGNET_HIST_BINS]
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const size_t tbase = (size_t)r * (size_t)T;
  WideEntry* const e = E + tbase;
  WideNode* const nd = ND + (size_t)r * (size_t)N;
  const bool hist = A.hist != nullptr;
  const int64_t arrive0 = T > 0 ? A.arrive[tbase] : kNever;

  // ---- node parameters + preconditions (fognet_hip.h, fognet_batch_in);
  // every node's first advert {MIPS, busyTime = 0.0} has reached the broker
  bool bad = false;
  for (int j = lane; j < N; j += kWave) {
    const int32_t m = A.mips[nbase + j];
    const int64_t d = A.dl[nbase + j], u = A.ul[nbase + j], ia = A.init[nbase + j];
    bad |= (m <= 0) | (d < 0) | (u < 0) | (d > kMaxTick) | (u > kMaxTick) | (ia < u) | (ia >= arrive0);
    if constexpr (kExt) bad |= d >= kExtMaxDl;
    s_nxt[j] = kNever;
    s_busy[j] = 0u;
    nd[j] = WideNode{-1, -1, 0, 0};
  }
  for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave) s_hist[h] = 0u;
  __syncthreads();
  uint32_t err = ballot(bad) ? (uint32_t)FOGNET_ERR_ARG : (uint32_t)FOGNET_OK;

  int64_t mn;
  int mj;
  uint64_t mk;
  lane_scan(s_nxt, s_busy, N, lane, mn, mj, mk);
  Acc acc = acc_identity();
  uint32_t max_pend = 0u;  // over this lane's nodes
  int64_t prev_t = INT64_MIN;
  int n_done = 0;

  for (int c0 = 0; c0 < T && err == FOGNET_OK; c0 += kWave) {
    const int cnt = min(kWave, T - c0);
    const bool live = lane < cnt;
    const int64_t ca = live ? A.arrive[tbase + c0 + lane] : kNever;
    const int32_t cr = live ? A.req[tbase + c0 + lane] : 0;
    // trace preconditions: nondecreasing ticks, requirement >= 0, ticks < 2^61
    const int64_t prv = dpp_or_i64<kDppWaveShr1>(prev_t, ca);  // lane 0 gets prev_t
    if (ballot(live && (ca < prv || cr < 0 || ca > kMaxTick))) {
      err = FOGNET_ERR_ARG;
      break;
    }
    prev_t = readlane_i64(ca, cnt - 1);

    for (int jp = 0; jp < cnt; ++jp) {
      const int64_t t = readlane_i64(ca, jp);
      const uint32_t rq = readlane_u32((uint32_t)cr, jp);

      // 1) completion adverts that reached the broker strictly before t
      bool lerr = false;
      while (ballot(mn < t)) {
        if (mn < t) {
          const int j = mj;
          lerr |= !apply_advert(j, nd, e, A.dl[nbase + j], A.ul[nbase + j], s_nxt, s_busy);
          lane_scan(s_nxt, s_busy, N, lane, mn, mj, mk);
        }
      }
      if (ballot(lerr)) {
        err = FOGNET_ERR_CAPACITY;
        break;
      }

      // 2) the decision over the advertised view
      uint32_t k;
      if constexpr (kExt) {
        // north-star cost (fognet_hip.h FOGNET_POLICY_EXT_LAT), first index on ties
        uint64_t mc = ~0ull;
        uint32_t mjj = ~0u;
        for (int j = lane; j < N; j += kWave) {
          const uint32_t S = min(rq / (uint32_t)A.mips[nbase + j], kExtSatS);
          const uint64_t c = (uint64_t)A.dl[nbase + j] + ((uint64_t)s_busy[j] + S) * (uint64_t)kTicksPerSecond;
          if (c < mc) {
            mc = c;
            mjj = (uint32_t)j;
          }
        }
        const uint64_t m = wave_min_u64(mc);
        k = wave_min_u32(mc == m ? mjj : ~0u);
      } else {
        // BrokerBaseApp3.cc:267-281: busy_j + req/mips_0 < tempp over exact
        // integer busy values <=> the smallest (busy, j)
        k = (uint32_t)wave_min_u64(mk);
      }

      // 3) node k: task arrival (ComputeBrokerApp3.cc:269-320), owner lane
      if (lane == (int)(k % kWave)) {
        WideNode h = nd[k];
        const int32_t mips_k = A.mips[nbase + k];
        const int64_t dl_k = A.dl[nbase + k], ul_k = A.ul[nbase + k];
        const uint32_t S = rq / (uint32_t)mips_k;  // double tskTime = requiredMIPS / MIPS (:276)
        const int64_t a = t + dl_k;
        int64_t prev_done = INT64_MIN;
        uint32_t prev_S = 0u;
        uint64_t prev_C = 0u;
        if (h.tl >= 0) {
          const WideEntry p = e[h.tl];
          prev_done = p.done;
          prev_S = p.S;
          prev_C = p.C;
        }
        const int64_t start = a > prev_done ? a : prev_done;
        const int64_t done = start + ticks_of(min(S, kWideMaxS));
        uint32_t status;
        if (prev_done < a) {
          status = 5u;  // idle: "task assigned" (:282-301)
        } else if (prev_done > a) {
          status = 4u;  // busy: "task queued" (:304-313)
        } else {        // the previous task completes at the same tick
          status = dl_k < (int64_t)prev_S * kTicksPerSecond ? 5u : 4u;
        }
        lerr = S > kWideMaxS || a > kMaxTick || done > kMaxTick;
        if (!lerr) {
          const int i = c0 + jp;
          e[i] = WideEntry{a, done, prev_C + S, S, h.tl, -1, 0};
          if (h.npend == 0) {
            h.hd = i;  // its completion advert is the node's next one
            const int64_t x = done + ul_k;
            s_nxt[k] = x;
            if (x < mn) {
              mn = x;
              mj = (int)k;
            }
          } else {
            e[h.tl].next = i;
          }
          h.tl = i;
          h.npend += 1;
          nd[k] = h;
          max_pend = max(max_pend, (uint32_t)h.npend);
          const size_t o = tbase + (size_t)i;
          A.out_node[o] = (int32_t)k;
          A.out_status[o] = (uint8_t)status;
          A.out_start[o] = start;
          A.out_done[o] = done;
          acc_task(acc, t, a, start, done, S, status);
          if (hist) {
            atomicAdd(&s_hist[FOGNET_HIST_BINS + hist_bin(done - t)], 1u);
            if (status == 4u) atomicAdd(&s_hist[hist_bin(start - a)], 1u);
          }
        }
      }
      if (ballot(lerr)) {
        err = FOGNET_ERR_ARG;
        break;
      }
      ++n_done;
    }
  }

  // ---- per-replication record (the fields replay_kernel + its epilogue write)
  acc = wave_merge(acc);
  const uint32_t mp = ~wave_min_u32(~max_pend);
  fognet_rep_stats* const S = A.out_stats + r;
  if (lane == 0 && A.out_stats) {
    S->n_tasks = n_done;
    S->max_pending = (int32_t)mp;
    S->status = (int32_t)err;
    S->events = 2 * (int64_t)N + 4 * (int64_t)n_done;
    write_rep_stats(S, acc);
  }
  // a11 energy (fognet_hip.h): E_j = P_busy_j * B_j + P_idle_j * ((H - B_j 1e12) / 1e12)
  // with B_j = node j's service seconds (its tail's cumulative sum), summed in node order
  if (A.p_busy && A.out_stats) {
    const int64_t H = n_done > 0 ? acc.last : 0;
    double* const s_e = reinterpret_cast<double*>(s_nxt);  // dead now; lane j%64 wrote s_nxt[j]
    for (int j = lane; j < N; j += kWave) {
      const int32_t tl = nd[j].tl;
      const int64_t B = tl >= 0 ? (int64_t)e[tl].C : 0;
      const double eb = __dmul_rn(A.p_busy[nbase + j], (double)B);
      const double idle = __ddiv_rn((double)(H - B * kTicksPerSecond), 1e12);
      const double en = __dadd_rn(eb, __dmul_rn(A.p_idle[nbase + j], idle));
      s_e[j] = en;
      if (A.out_energy) A.out_energy[(size_t)r * (size_t)N + j] = en;
    }
    __syncthreads();
    if (lane == 0) {
      double sum = 0.0;
      for (int j = 0; j < N; ++j) sum = __dadd_rn(sum, s_e[j]);
      S->energy_j = sum;
    }
  }
  if (hist) {
    __syncthreads();
    for (int h = lane; h < FOGNET_HIST_METRICS * FOGNET_HIST_BINS; h += kWave)
      if (s_hist[h]) atomicAdd((unsigned long long*)&A.hist[h], (unsigned long long)s_hist[h]);
  }
}

template <int POL>
void launch_wide_pol(const ReplayArgs& a, WideEntry* e, WideNode* nd, size_t lds, hipStream_t s) {
  // dynamic LDS above 64 KiB (a single workgroup may take all 160 KiB on gfx950)
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&replay_wide_kernel<POL>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  (void)hipGetLastError();
  hipLaunchKernelGGL((replay_wide_kernel<POL>), dim3(a.R), dim3(kWave), lds, s, a, e, nd);
}

}  // namespace

size_t replay_wide_lds_bytes(int32_t N) {
  return (size_t)N * (sizeof(int64_t) + sizeof(uint32_t)) + FOGNET_HIST_METRICS * FOGNET_HIST_BINS * sizeof(uint32_t);
}

size_t replay_wide_workspace_bytes(int32_t R, int32_t T, int32_t N) {
  return (size_t)R * (size_t)T * sizeof(WideEntry) + (size_t)R * (size_t)N * sizeof(WideNode);
}

hipError_t launch_replay_wide(const ReplayArgs& a, void* workspace, hipStream_t s) {
  WideEntry* const e = reinterpret_cast<WideEntry*>(workspace);
  WideNode* const nd = reinterpret_cast<WideNode*>(e + (size_t)a.R * (size_t)a.T);
  const size_t lds = replay_wide_lds_bytes(a.N);
  if (a.policy == FOGNET_POLICY_EXT_LAT)
    launch_wide_pol<FOGNET_POLICY_EXT_LAT>(a, e, nd, lds, s);
  else
    launch_wide_pol<FOGNET_POLICY_REF_V3>(a, e, nd, lds, s);
  return hipGetLastError();
}

}  // namespace fognet
