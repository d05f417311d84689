// decide.hip — M independent broker decisions: BrokerBaseApp3.cc:265-281
// (decide_kernel) and BrokerBaseApp2.cc:180-192/235-286 (decide_v2_kernel).
// The v3 core is evaluated with the reference's exact arithmetic:
//   tskTime = req / brokers[0].MIPS           (int / int, then double)
//   tempp   = busy[0] + tskTime
//   for j in 0..n-1: if busy[j] + tskTime < tempp: tempp = ..., k = j   (strict '<')
// The sequential scan returns the first index attaining the minimum of
// c_j = busy_j + tskTime among non-NaN c_j, or 0 when c_0 is NaN (no
// comparison against a NaN tempp is ever true).  One wavefront per query; the
// lanes scan strided candidates and a (value, index) reduction keeps the
// earliest index on ties, which reproduces the sequential result exactly.
#include "internal.h"

namespace fognet {

namespace {

constexpr int kDecideThreads = 256;  // 4 queries per workgroup

struct Cand {
  double c;
  int32_t j;
};

// a precedes b in the scan's outcome
__device__ __forceinline__ bool better(const Cand& a, const Cand& b) {
  if (a.j < 0) return false;
  if (b.j < 0) return true;
  return a.c < b.c || (a.c == b.c && a.j < b.j);
}

// One decision by one wavefront: rc / out as the reference's scan
// (busy: the advertised view b[0..n), mips0 = brokers[0]->getMips()).
template <class Busy>
__device__ __forceinline__ void decide_one(int32_t n, Busy b, int32_t m0, int32_t rq, int lane, int32_t& out,
                                           int32_t& rc) {
  rc = FOGNET_OK;
  out = -1;
  if (n <= 0) {
    rc = FOGNET_ERR_NO_NODES;
  } else if (m0 == 0) {
    rc = FOGNET_ERR_DIV0;
  } else if (m0 == -1 && rq == INT32_MIN) {
    rc = FOGNET_ERR_ARG;  // INT_MIN / -1 overflows in the reference
  } else {
    const double tsk = (double)(rq / m0);
    const double c0 = b(0) + tsk;
    if (c0 != c0) {
      out = 0;  // tempp is NaN: no candidate can replace node 0
    } else {
      Cand best = {0.0, -1};
      for (int32_t j = lane; j < n; j += kWave) {
        const double c = b(j) + tsk;
        if (c == c) {
          const Cand cj = {c, j};
          if (better(cj, best)) best = cj;
        }
      }
      // wave reduction, butterfly over xor distances
      for (int off = 32; off > 0; off >>= 1) {
        Cand o;
        o.c = __shfl_xor(best.c, off);
        o.j = __shfl_xor(best.j, off);
        if (better(o, best)) best = o;
      }
      out = best.j;  // node 0 is a non-NaN candidate, so best.j >= 0
    }
  }
}

// view_stride: n (one view per query) or 0 (one view shared by all queries:
// the publishes of one window between two adverts, fognet_decide_window).
__global__ __launch_bounds__(kDecideThreads) void decide_kernel(int64_t m, int32_t n, int64_t view_stride,
                                                                 const double* busy, const int32_t* mips,
                                                                 const int32_t* req, int32_t* node, int32_t* status) {
  const int64_t q = (int64_t)blockIdx.x * (kDecideThreads / kWave) + threadIdx.x / kWave;
  const int lane = threadIdx.x % kWave;
  if (q >= m) return;  // whole wave exits together
  int32_t rc, out;
  const double* b = busy + q * view_stride;
  decide_one(n, [&](int32_t j) { return b[j]; }, n > 0 ? mips[q * view_stride] : 0, req[q], lane, out, rc);
  if (lane == 0) {
    node[q] = out;
    if (status) status[q] = rc;
  }
}

// The scalar drop-in (fognet_decide): the view travels in the kernel
// arguments (n <= kDecideArgNodes) or is read from mapped host memory, and the
// result is written straight to mapped host memory: one launch and one stream
// synchronisation per decision, no copies.
__global__ __launch_bounds__(kWave) void decide_arg_kernel(DecideArgs a, const double* far_busy, int32_t* res) {
  int32_t rc, out;
  if (a.n <= kDecideArgNodes)
    decide_one(a.n, [&](int32_t j) { return a.busy[j]; }, a.mips0, a.req, threadIdx.x, out, rc);
  else
    decide_one(a.n, [&](int32_t j) { return far_busy[j]; }, a.mips0, a.req, threadIdx.x, out, rc);
  if (threadIdx.x == 0) {
    res[0] = out;
    res[1] = rc;
    __threadfence_system();
  }
}

// BrokerBaseApp2 (BrokerBaseApp2.cc:180-192, 235-286): one wavefront per
// query.  The reference's loop takes index i+1 whenever brokers[i+1].MIPS >
// brokers[0].MIPS (temp is never updated), i.e. the LAST such index; the lanes
// scan strided candidates and a wave max keeps the largest qualifying index.
__global__ __launch_bounds__(kDecideThreads) void decide_v2_kernel(int64_t m, int32_t n, const int32_t* mips,
                                                                    const int32_t* local, const int32_t* req,
                                                                    int32_t* node, int32_t* action) {
  const int64_t q = (int64_t)blockIdx.x * (kDecideThreads / kWave) + threadIdx.x / kWave;
  const int lane = threadIdx.x % kWave;
  if (q >= m) return;  // whole wave exits together
  const int32_t rq = req[q];
  int32_t out = -1, act;
  if (rq < local[q]) {
    act = FOGNET_V2_LOCAL;  // :181
  } else if (n <= 0) {
    act = FOGNET_V2_NO_NODES;  // :273-285
  } else {
    const int32_t* v = mips + q * (int64_t)n;
    const int32_t temp = v[0];  // :241
    uint32_t last = 0u;         // currentGoodBroker = 0 (:237)
    for (int32_t j = 1 + lane; j < n; j += kWave)
      if (v[j] > temp) last = (uint32_t)j;  // ascending per lane: keeps the lane's largest
    out = (int32_t)~wave_min_u32(~last);
    act = rq < v[out] ? FOGNET_V2_FORWARD : FOGNET_V2_DROPPED;  // :262
  }
  if (lane == 0) {
    node[q] = out;
    action[q] = act;
  }
}

}  // namespace

hipError_t launch_decide_v2(int64_t m, int32_t n, const int32_t* mips, const int32_t* local, const int32_t* req,
                            int32_t* node, int32_t* action, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int per = kDecideThreads / kWave;
  const int64_t blocks = (m + per - 1) / per;
  hipLaunchKernelGGL(decide_v2_kernel, dim3((unsigned)blocks), dim3(kDecideThreads), 0, s, m, n, mips, local, req,
                     node, action);
  return hipGetLastError();
}

hipError_t launch_decide(int64_t m, int32_t n, int64_t view_stride, const double* busy, const int32_t* mips,
                         const int32_t* req, int32_t* node, int32_t* status, hipStream_t s) {
  if (m <= 0) return hipSuccess;
  const int per = kDecideThreads / kWave;
  const int64_t blocks = (m + per - 1) / per;
  hipLaunchKernelGGL(decide_kernel, dim3((unsigned)blocks), dim3(kDecideThreads), 0, s, m, n, view_stride, busy, mips,
                     req, node, status);
  return hipGetLastError();
}

hipError_t launch_decide_args(const DecideArgs& a, const double* far_busy, int32_t* res, hipStream_t s) {
  hipLaunchKernelGGL(decide_arg_kernel, dim3(1), dim3(kWave), 0, s, a, far_busy, res);
  return hipGetLastError();
}

}  // namespace fognet
