// user_stats.hip — the user-side signals of the offload loop, computed on the
// device from a finished replay (fognet_user_stats_dev).
//
// The reference's acks: the broker's own status-4 pubAck at the publish
// (BrokerBaseApp3.cc:145-150), the node's status 5/4 at the task's arrival
// (ComputeBrokerApp3.cc:284-289, 310-313) and status 6 at its completion
// (:228-233); node acks reach the broker one uplink later and are relayed
// (BrokerBaseApp3.cc:164-198) to the user, one user downlink later.  The user
// emits (simTime() - created) * 1000 for each (mqttApp2.cc:252-291; raw
// simtime_t values, fognet_hip.h "Reference signal values"), created = the
// publish's send time = its broker arrival - the user uplink.  Acks carry no
// state back into the decision loop, so every signal is a closed form of the
// replay outputs; tests/oracle_lib restates them as real FES events.
// Memory-bound: one 256-thread workgroup per replication streams its tasks.
#include "replay_common.h"

namespace fognet {

namespace {

constexpr int kUserThreads = 256;
constexpr int kSignals = 4;  // delay, latency, latencyH1, taskTime

// moments of raw emitted values (fognet_hip.h "Reference signal values")
struct Mom {
  uint64_t n, s_lo, s_hi, q_lo, q_hi, q_top, ovf;
  int64_t mn, mx;
};

__device__ __forceinline__ void mom_init(Mom& m) {
  m = Mom{0u, 0u, 0u, 0u, 0u, 0u, 0u, INT64_MAX, INT64_MIN};
}

__device__ __forceinline__ void mom_add(Mom& m, int64_t raw) {
  m.n += 1u;
  add_moment_signed(m.s_lo, m.s_hi, m.q_lo, m.q_hi, m.q_top, raw);
  m.mn = min(m.mn, raw);
  m.mx = max(m.mx, raw);
}

// emit(signal, (simTime() - created) * 1000) (mqttApp2.cc:260,272,282); an
// overflowing product throws and mqttApp2's catch drops the emission
__device__ __forceinline__ void mom_add_ms(Mom& m, int64_t d) {
  int64_t raw;
  if (ms_raw(d, raw)) mom_add(m, raw);
  else m.ovf += 1u;
}

__device__ __forceinline__ void mom_merge(Mom& a, const Mom& b) {
  a.n += b.n;
  a.ovf += b.ovf;
  add128(a.s_lo, a.s_hi, b.s_lo, b.s_hi);
  add192(a.q_lo, a.q_hi, a.q_top, b.q_lo, b.q_hi, b.q_top);
  a.mn = min(a.mn, b.mn);
  a.mx = max(a.mx, b.mx);
}

__global__ __launch_bounds__(kUserThreads) void user_stats_kernel(ReplayArgs A, const int64_t* uul, const int64_t* udl,
                                                                  int32_t per_task, fognet_user_stats* out) {
  __shared__ Mom sh[kUserThreads];
  const int r = blockIdx.x;
  const size_t tbase = (size_t)r * (size_t)A.T;
  const size_t nbase = (size_t)r * (size_t)A.node_stride;
  const int n = (int)A.out_stats[r].n_tasks;  // decided tasks (written by the replay)
  Mom m[kSignals];
  for (int s = 0; s < kSignals; ++s) mom_init(m[s]);
  for (int i = threadIdx.x; i < n; i += kUserThreads) {
    const size_t o = tbase + (size_t)i;
    const int64_t t = A.arrive[o];
    const int k = A.out_node[o];
    const uint32_t st = A.out_status[o];
    const int64_t done = A.out_done[o];
    const size_t uo = per_task ? o : (size_t)r;
    const int64_t uu = uul[uo], ud = udl[uo];
    const int64_t created = t - uu;
    const int64_t relay = A.ul[nbase + k] + ud;  // node -> broker -> user
    mom_add(m[0], uu);                            // delay: at the broker (:143), a simtime_t (s)
    mom_add_ms(m[2], t + ud - created);           // broker pubAck status 4 -> latencyH1
    const int64_t at_arrival = t + A.dl[nbase + k] + relay - created;  // node ack sent at the task's arrival
    if (st == 5u)
      mom_add_ms(m[1], at_arrival);  // "task assigned" -> latency
    else if (st == 4u)
      mom_add_ms(m[2], at_arrival);  // "task queued" -> latencyH1
    // (status 9: the task reached a crashed node, which sends no ack)
    if (done >= 0) mom_add_ms(m[3], done + relay - created);  // status 6 -> taskTime (-1: never completed)
  }
  fognet_moments* dst[kSignals] = {&out[r].delay, &out[r].latency, &out[r].latencyH1, &out[r].taskTime};
  for (int s = 0; s < kSignals; ++s) {
    sh[threadIdx.x] = m[s];
    __syncthreads();
    for (int w = kUserThreads / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) mom_merge(sh[threadIdx.x], sh[threadIdx.x + w]);
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const Mom& b = sh[0];
      *dst[s] = fognet_moments{(int64_t)b.n, b.mn, b.mx, b.s_lo, b.s_hi, b.q_lo, b.q_hi, b.q_top, (int64_t)b.ovf};
    }
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_user_stats(const ReplayArgs& a, const int64_t* user_ul, const int64_t* user_dl, int32_t per_task,
                             fognet_user_stats* out, hipStream_t s) {
  if (a.R <= 0) return hipSuccess;
  hipLaunchKernelGGL(user_stats_kernel, dim3(a.R), dim3(kUserThreads), 0, s, a, user_ul, user_dl, per_task, out);
  return hipGetLastError();
}

}  // namespace fognet
