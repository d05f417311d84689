// tracegen.hip — device generator for the synthetic trace-replay workloads
// (SURVEY.md §8(d) C2/C3).  Integer-exact recipe shared with the host
// restatement tests/tracegen.py (which documents it):
//   replication r: Philox4x32-10 key (seed, r)
//   node j:  counter (j, 1, 0, 0) -> dl, ul ~ U_int[1e6, 1e9] * lat_scale[r];
//            mips = 1000 * (1 + j % 4); first advert arrives at init = ul
//   task i:  counter (i, 0, 0, 0) -> req ~ U_int[req_lo, req_hi],
//            u = ((x1 << 21 | x2 >> 11) + 1) * 2^-53, gap = trunc(mean_gap * -ln u)
//            arrive[0] = max(init) + 1 + gap[0], arrive[i] = arrive[i-1] + gap[i]
#include "internal.h"

namespace fognet {

namespace {

constexpr int kGenThreads = 256;

__device__ __forceinline__ int64_t block_max_i64(int64_t v, int64_t* sh) {
  for (int off = 32; off > 0; off >>= 1) {
    const int64_t o = __shfl_xor(v, off);
    v = o > v ? o : v;
  }
  if (threadIdx.x % kWave == 0) sh[threadIdx.x / kWave] = v;
  __syncthreads();
  int64_t m = sh[0];
  for (int w = 1; w < kGenThreads / kWave; ++w) m = sh[w] > m ? sh[w] : m;
  __syncthreads();
  return m;
}

// inclusive scan of int64 over the block
__device__ __forceinline__ int64_t block_scan_i64(int64_t v, int64_t* sh) {
  const int lane = threadIdx.x % kWave, w = threadIdx.x / kWave;
  for (int off = 1; off < kWave; off <<= 1) {
    const int64_t o = __shfl_up(v, off);
    if (lane >= off) v += o;
  }
  if (lane == kWave - 1) sh[w] = v;
  __syncthreads();
  int64_t pre = 0;
  for (int i = 0; i < w; ++i) pre += sh[i];
  __syncthreads();
  return v + pre;
}

__global__ __launch_bounds__(kGenThreads) void gen_kernel(fognet_gen_params p, int64_t r0, int32_t T, int32_t N,
                                                          int64_t* arrive, int32_t* req, int32_t* mips,
                                                          int64_t* dl, int64_t* ul, int64_t* init) {
  __shared__ int64_t sh[kGenThreads / kWave];
  const int rl = blockIdx.x;  // local replication index
  const int64_t r = r0 + rl;
  const GenRep g = gen_rep(p, r, rl);
  int64_t my_max = INT64_MIN;
  for (int j = threadIdx.x; j < N; j += kGenThreads) {
    int32_t m;
    int64_t d, u;
    gen_node(g, j, m, d, u);
    const size_t o = (size_t)rl * N + j;
    dl[o] = d;
    ul[o] = u;
    init[o] = u;
    mips[o] = m;
    my_max = u > my_max ? u : my_max;
  }
  const int64_t start = block_max_i64(my_max, sh) + 1;
  int64_t carry = start;
  for (int base = 0; base < T; base += kGenThreads) {
    const int i = base + threadIdx.x;
    int64_t gap = 0;
    int32_t rq = 0;
    if (i < T) gen_task(g, i, gap, rq);
    const int64_t inc = block_scan_i64(gap, sh);
    if (i < T) {
      const size_t o = (size_t)rl * T + i;
      arrive[o] = carry + inc;
      req[o] = rq;
    }
    // carry += sum of this block's gaps (the last thread's inclusive value)
    if (threadIdx.x == kGenThreads - 1) sh[0] = inc;
    __syncthreads();
    carry += sh[0];
    __syncthreads();
  }
}

// ---------------------------------------------------------------- job stats

constexpr int kRedThreads = 256;

__device__ __forceinline__ void add192(uint64_t* a, uint64_t lo, uint64_t mid, uint64_t hi) {
  uint64_t o = a[0];
  a[0] += lo;
  uint64_t c = a[0] < o ? 1u : 0u;
  o = a[1];
  a[1] += mid;
  uint64_t c2 = a[1] < o ? 1u : 0u;
  o = a[1];
  a[1] += c;
  c2 += a[1] < o ? 1u : 0u;
  a[2] += hi + c2;
}

__device__ __forceinline__ void job_init(fognet_job_stats& j) {
  j = fognet_job_stats{};
  j.queue_min_raw = j.resp_min_ticks = INT64_MAX;
  j.queue_max_raw = j.resp_max_ticks = j.last_tick = INT64_MIN;
}

__device__ __forceinline__ void job_merge(fognet_job_stats& a, const fognet_job_stats& b) {
  a.n_reps += b.n_reps;
  a.n_failed += b.n_failed;
  a.n_tasks += b.n_tasks;
  a.n_queued += b.n_queued;
  a.n_started += b.n_started;
  a.events += b.events;
  a.last_tick = max(a.last_tick, b.last_tick);
  a.queue_min_raw = min(a.queue_min_raw, b.queue_min_raw);
  a.queue_max_raw = max(a.queue_max_raw, b.queue_max_raw);
  a.n_qtime += b.n_qtime;
  a.n_qtime_overflow += b.n_qtime_overflow;
  a.n_ref_aborted += b.n_ref_aborted;
  a.resp_min_ticks = min(a.resp_min_ticks, b.resp_min_ticks);
  a.resp_max_ticks = max(a.resp_max_ticks, b.resp_max_ticks);
  a.max_pending = max(a.max_pending, b.max_pending);
  a.busy_s += b.busy_s;
  a.energy_j = __dadd_rn(a.energy_j, b.energy_j);
  add192(a.queue_sum, b.queue_sum[0], b.queue_sum[1], b.queue_sum[2]);
  add192(a.queue_sq, b.queue_sq[0], b.queue_sq[1], b.queue_sq[2]);
  add192(a.resp_sum, b.resp_sum[0], b.resp_sum[1], b.resp_sum[2]);
  add192(a.resp_sq, b.resp_sq[0], b.resp_sq[1], b.resp_sq[2]);
}

// Block b reduces records [b * chunk, min(R, (b + 1) * chunk)) into out[b].
__global__ __launch_bounds__(kRedThreads) void reduce_kernel(const fognet_rep_stats* st, int32_t R, int32_t chunk,
                                                             fognet_job_stats* out) {
  __shared__ fognet_job_stats sh[kRedThreads];
  fognet_job_stats a;
  job_init(a);
  const int r0 = blockIdx.x * chunk, r1 = min(R, r0 + chunk);
  for (int r = r0 + threadIdx.x; r < r1; r += kRedThreads) {
    const fognet_rep_stats& s = st[r];
    a.n_reps += 1;
    // the reference's abort point counts under FOGNET_FLAG_REF_ABORT too, where such a replication's
    // status is FOGNET_REF_ABORTED (failed: it contributes nothing else)
    if (s.status == FOGNET_OK || s.status == FOGNET_REF_ABORTED) a.n_ref_aborted += s.abort_tick != INT64_MAX ? 1 : 0;
    if (s.status != FOGNET_OK) {
      a.n_failed += 1;
      continue;
    }
    a.n_tasks += s.n_tasks;
    a.n_queued += s.n_queued;
    a.n_started += s.n_started;
    a.events += s.events;
    a.last_tick = max(a.last_tick, s.last_tick);
    a.queue_min_raw = min(a.queue_min_raw, s.queue_min_raw);
    a.queue_max_raw = max(a.queue_max_raw, s.queue_max_raw);
    a.n_qtime += s.n_qtime;
    a.n_qtime_overflow += s.n_qtime_overflow;
    a.resp_min_ticks = min(a.resp_min_ticks, s.resp_min_ticks);
    a.resp_max_ticks = max(a.resp_max_ticks, s.resp_max_ticks);
    a.max_pending = max(a.max_pending, (int64_t)s.max_pending);
    a.busy_s += s.busy_s;
    a.energy_j = __dadd_rn(a.energy_j, s.energy_j);
    add192(a.queue_sum, s.queue_sum_lo, s.queue_sum_hi, (int64_t)s.queue_sum_hi < 0 ? ~(uint64_t)0 : 0u);  // signed
    add192(a.queue_sq, s.queue_sq_lo, s.queue_sq_hi, s.queue_sq_top);
    add192(a.resp_sum, s.resp_sum_lo, s.resp_sum_hi, 0u);
    add192(a.resp_sq, s.resp_sq_lo, s.resp_sq_hi, 0u);
  }
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int w = kRedThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) job_merge(sh[threadIdx.x], sh[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0];
}

// Merge of n partial job records (the blocks of reduce_kernel), in the same tree shape.
__global__ __launch_bounds__(kRedThreads) void merge_jobs_kernel(const fognet_job_stats* parts, int32_t n,
                                                                 fognet_job_stats* out) {
  __shared__ fognet_job_stats sh[kRedThreads];
  fognet_job_stats a;
  job_init(a);
  for (int i = threadIdx.x; i < n; i += kRedThreads) job_merge(a, parts[i]);
  sh[threadIdx.x] = a;
  __syncthreads();
  for (int w = kRedThreads / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) job_merge(sh[threadIdx.x], sh[threadIdx.x + w]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

}  // namespace

hipError_t launch_gen_trace(const fognet_gen_params& p, int64_t r0, int32_t R, int32_t T, int32_t N,
                            int64_t* arrive, int32_t* req, int32_t* mips, int64_t* dl, int64_t* ul,
                            int64_t* init, hipStream_t s) {
  if (R <= 0) return hipSuccess;
  hipLaunchKernelGGL(gen_kernel, dim3(R), dim3(kGenThreads), 0, s, p, r0, T, N, arrive, req, mips, dl, ul, init);
  return hipGetLastError();
}

int32_t reduce_stats_parts(int32_t R) { return R <= kReduceChunk ? 0 : (R + kReduceChunk - 1) / kReduceChunk; }

hipError_t launch_reduce_stats(const fognet_rep_stats* st, int32_t R, fognet_job_stats* out, fognet_job_stats* parts,
                               hipStream_t s) {
  const int32_t np = reduce_stats_parts(R);
  if (np == 0) {  // one block (up to kReduceChunk records)
    hipLaunchKernelGGL(reduce_kernel, dim3(1), dim3(kRedThreads), 0, s, st, R, R, out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(reduce_kernel, dim3(np), dim3(kRedThreads), 0, s, st, R, kReduceChunk, parts);
  hipLaunchKernelGGL(merge_jobs_kernel, dim3(1), dim3(kRedThreads), 0, s, parts, np, out);
  return hipGetLastError();
}

}  // namespace fognet
