// capi.hip — host implementation of the libfognet_hip C ABI (include/fognet_hip.h).
// Pure host C++ around the gfx950 kernels; there is no CPU compute path: every
// decision is evaluated on the device, and the library refuses to create a
// context without a gfx950 GPU.
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "internal.h"

struct fognet_ctx {
  int device = -1;
  int cus = 256;  // compute units (generated-mode launch size)
  hipStream_t stream = nullptr;  // private stream for the host-buffer entry points
  fognet::RingWord* ring = nullptr;
  size_t ring_bytes = 0;
  // partial job records of a multi-block reduction (fognet_reduce_stats_dev)
  void* red = nullptr;
  size_t red_bytes = 0;
  // scratch for the v2 scalar decision
  void* scratch = nullptr;
  size_t scratch_bytes = 0;
  // mapped, coherent host memory for fognet_decide / fognet_decide_window:
  // inputs the kernel reads and results it writes without copies
  void* host_stage = nullptr;
  void* host_stage_dev = nullptr;
  size_t host_stage_bytes = 0;
  // EXT_HIER path choice (fognet_hier_path_stats): the hand-over count of the last region pass,
  // copied back into pinned memory on the launch stream and read once its event has passed
  // One measurement at a time: the count is paired with the shape and stream of the
  // launch it measured, and its decision applies only to later launches of that same shape and stream.
  struct HierShape {
    int32_t R, T, N;
    void* stream;
    bool operator==(const HierShape& o) const { return R == o.R && T == o.T && N == o.N && stream == o.stream; }
  };
  int32_t* hier_host = nullptr;  // [0] handed-over replications of the measured launch
  hipEvent_t hier_ev = nullptr;
  bool hier_pending = false;
  HierShape hier_pend_shape{};  // the launch being measured
  bool hier_seq = false;  // the last measured region pass (of hier_seq_shape) handed most replications over
  HierShape hier_seq_shape{};
  int hier_seq_runs = 0;  // launches sent straight to the sequential replay since that measurement
  int64_t hier_region_launches = 0, hier_seq_launches = 0;
  std::string err;
};

namespace {

constexpr int kDefaultRing = 2048;
// Workspace slots of the wide kernel when it replays the replications the
// register kernel hands over (at most one wave per SIMD of the chip).
constexpr int32_t kWideFallbackSlots = 1024;

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

int fail(fognet_ctx* c, int rc, const std::string& msg) {
  if (c) c->err = msg;
  return rc;
}

int hip_fail(fognet_ctx* c, hipError_t e, const char* what) {
  return fail(c, FOGNET_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(fognet_ctx* c, void** p, size_t* have, size_t want, const char* what) {
  if (*have >= want) return FOGNET_OK;
  if (*p) {
    (void)hipFree(*p);
    *p = nullptr;
    *have = 0;
  }
  hipError_t e = hipMalloc(p, want);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(c, e == hipErrorOutOfMemory ? FOGNET_ERR_OOM : FOGNET_ERR_DEVICE,
                std::string("hipMalloc ") + what + ": " + hipGetErrorString(e));
  }
  *have = want;
  return FOGNET_OK;
}

int ensure_host(fognet_ctx* c, size_t want) {
  if (c->host_stage_bytes >= want) return FOGNET_OK;
  if (c->host_stage) {
    (void)hipHostFree(c->host_stage);
    c->host_stage = c->host_stage_dev = nullptr;
    c->host_stage_bytes = 0;
  }
  want = want < 4096 ? 4096 : want;
  hipError_t e = hipHostMalloc(&c->host_stage, want, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) e = hipHostGetDevicePointer(&c->host_stage_dev, c->host_stage, 0);
  if (e != hipSuccess) {
    if (c->host_stage) (void)hipHostFree(c->host_stage);
    c->host_stage = c->host_stage_dev = nullptr;
    return fail(c, FOGNET_ERR_OOM, std::string("hipHostMalloc decide stage: ") + hipGetErrorString(e));
  }
  c->host_stage_bytes = want;
  return FOGNET_OK;
}

int set_device(fognet_ctx* c) {
  hipError_t e = hipSetDevice(c->device);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "hipSetDevice");
}

// Validates a batch descriptor; fills the kernel argument block except pointers to outputs.
// generated: fognet_run_generated_dev (no trace or node-parameter arrays)
int prepare(fognet_ctx* c, const fognet_batch_in* in, fognet::ReplayArgs* a, bool generated = false) {
  if (!in) return fail(c, FOGNET_ERR_ARG, "null batch");
  if (in->R < 0 || in->T < 0 || in->N < 0) return fail(c, FOGNET_ERR_ARG, "negative R/T/N");
  if (in->N == 0) return fail(c, FOGNET_ERR_NO_NODES, "N == 0 (BrokerBaseApp3.cc:268 reads brokers[0])");
  if (in->N > fognet::kWideBigMaxNodes)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "N > 1048576 (the wide replay kernel's active-group mask: 16 words per lane)");
  if (in->policy == FOGNET_POLICY_EXT_HIER && in->N > fognet::kWideMaxNodes)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "EXT_HIER with N > 65536 (more than 64 regions of 1,024 nodes)");
  if (in->policy != FOGNET_POLICY_REF_V3 && in->policy != FOGNET_POLICY_EXT_LAT && in->policy != FOGNET_POLICY_EXT_HIER)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "unknown policy");
  if (in->policy == FOGNET_POLICY_EXT_HIER) {
    if (!generated && in->R > 0 && in->T > 0 && !in->region) return fail(c, FOGNET_ERR_ARG, "EXT_HIER needs the region array");
    if (in->hier_threshold_s < 0 || in->hier_up_tick < 0 || in->hier_up_tick >= ((int64_t)1 << 50))
      return fail(c, FOGNET_ERR_ARG, "EXT_HIER: threshold >= 0 and 0 <= up latency < 2^50 ticks");
  }
  if ((in->p_busy_w == nullptr) != (in->p_idle_w == nullptr))
    return fail(c, FOGNET_ERR_ARG, "p_busy_w and p_idle_w must both be given or both be null");
  if (in->down_tick && in->p_busy_w)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "the power model assumes nodes that stay up (down_tick with p_busy_w)");
  if (in->node_stride != 0 && in->node_stride != in->N)
    return fail(c, FOGNET_ERR_ARG, "node_stride must be 0 or N");
  if (in->flags & ~FOGNET_FLAG_REF_ABORT) return fail(c, FOGNET_ERR_ARG, "unknown flags");
  int q = in->ring_capacity ? in->ring_capacity : kDefaultRing;
  if (q < 2 || (q & (q - 1)) != 0 || q > (1 << 15)) return fail(c, FOGNET_ERR_ARG, "ring_capacity must be a power of two in [2, 2^15]");
  int qlog = 0;
  while ((1 << qlog) < q) ++qlog;
  if (!generated && in->R > 0 && in->T > 0 && (!in->arrive_tick || !in->req_mips))
    return fail(c, FOGNET_ERR_ARG, "null trace arrays");
  if (!generated && in->R > 0 && (!in->mips || !in->dl_tick || !in->ul_tick || !in->init_adv_tick))
    return fail(c, FOGNET_ERR_ARG, "null node parameter arrays");
  memset(a, 0, sizeof *a);
  a->R = in->R;
  a->T = in->T;
  a->N = in->N;
  a->node_stride = in->node_stride;
  a->q_log2 = qlog;
  // busy (a sum of at most Q pending service times) must stay below 2^24 s
  // (the replay kernel's 32-bit view key is busy << 8 | node), and service
  // times stay below 2^16 s (18.2 h) so its run scan cannot overflow
  // (replay.hip, kMaxTick).  Q = 1024: at most 16383 s per task.
  const uint64_t by_ring = 0xFFFFFFull / (uint64_t)q;
  a->max_s = (uint32_t)(by_ring < 0xFFFFull ? by_ring : 0xFFFFull);
  a->arrive = in->arrive_tick;
  a->req = in->req_mips;
  a->mips = in->mips;
  a->dl = in->dl_tick;
  a->ul = in->ul_tick;
  a->init = in->init_adv_tick;
  a->policy = in->policy;
  a->p_busy = in->p_busy_w;
  a->p_idle = in->p_idle_w;
  a->down = in->down_tick;
  a->ref_abort = (in->flags & FOGNET_FLAG_REF_ABORT) ? 1 : 0;
  if (in->policy == FOGNET_POLICY_EXT_HIER) {
    a->region = in->region;
    a->hier_up = in->hier_up_tick;
    a->hier_thr = in->hier_threshold_s;
  }
  return FOGNET_OK;
}

// N > 256 takes the wide replay kernel (replay_wide.hip); FOGNET_REPLAY_KERNEL=wide
// forces it for any N (used by the parity tests to check both kernels).
// FOGNET_REPLAY_STATS=inloop: the statistics of a fused replay come from
// in-loop accumulators (replay_inl_kernel, 3 waves/SIMD) instead of the
// epilogue's re-read of the outputs (replay_kernel, 4 waves/SIMD); the records
// are identical (the parity tests run both).  Not the default: at C3 (4,096
// replications, all resident at 4 waves/SIMD) it measured 20.9 ms/launch
// against 14.1 ms, the fourth wave per SIMD being worth more than the re-read.
// FOGNET_HIER_REGIONS=0: EXT_HIER replays run on the sequential wide kernel
// only; =only: the region pass without the sequential hand-over (a replication
// it cannot finish keeps an internal status) -- the parity tests use both to
// check that each path ran.
bool use_regions() {
  const char* f = getenv("FOGNET_HIER_REGIONS");
  return f == nullptr || strcmp(f, "0") != 0;
}
bool regions_auto() { return getenv("FOGNET_HIER_REGIONS") == nullptr; }
// FOGNET_HIER_RESUME=0: an escalated replication is replayed by the sequential kernel from the
// start (and the automatic mode below chooses between the two paths); default: it continues from
// its first escalated publish (replay_region.hip)
bool use_resume() {
  const char* f = getenv("FOGNET_HIER_RESUME");
  return f == nullptr || strcmp(f, "0") != 0;
}
// automatic mode: after a region pass that handed most replications over, this many launches go
// straight to the sequential replay before a region pass measures again
constexpr int kHierReprobe = 15;
bool regions_only() {
  const char* f = getenv("FOGNET_HIER_REGIONS");
  return f != nullptr && strcmp(f, "only") == 0;
}

bool use_inloop() {
  const char* f = getenv("FOGNET_REPLAY_STATS");
  return f != nullptr && strcmp(f, "inloop") == 0;
}

// Workspace slots of the hand-over launch: the wide kernel walks the hand-over
// list with a grid stride, so fewer slots than handed-over replications are
// still exact.  At most kWideFallbackSlots, and no more than fit in the ring
// workspace the register kernel needs anyway (floor 1), so a replay that never
// hands over allocates nothing extra.
int32_t fallback_slots(int32_t R, int32_t T, int32_t N, size_t ring_bytes, bool gen, int policy) {
  int32_t slots = R < kWideFallbackSlots ? R : kWideFallbackSlots;
  const size_t per = fognet::replay_wide_workspace_bytes(1, T, N, gen, policy);
  const size_t fit = per ? ring_bytes / per : (size_t)slots;
  if ((size_t)slots > fit) slots = fit < 1 ? 1 : (int32_t)fit;
  return slots;
}

bool use_wide(int32_t N) {
  if (N > fognet::kWave * fognet::kMaxNodesPerLane) return true;
  const char* f = getenv("FOGNET_REPLAY_KERNEL");
  return f != nullptr && strcmp(f, "wide") == 0;
}

}  // namespace

extern "C" {

int fognet_abi_version(void) { return FOGNET_ABI_VERSION; }

const char* fognet_status_string(int s) {
  switch (s) {
    case FOGNET_OK: return "ok";
    case FOGNET_ERR_ARG: return "invalid argument";
    case FOGNET_ERR_NO_NODES: return "no fog nodes registered";
    case FOGNET_ERR_DIV0: return "advertised MIPS of node 0 is zero";
    case FOGNET_ERR_STATE: return "self-message already scheduled";
    case FOGNET_ERR_DEVICE: return "HIP device error";
    case FOGNET_ERR_OOM: return "out of device memory";
    case FOGNET_ERR_CAPACITY: return "capacity exceeded";
    case FOGNET_ERR_UNSUPPORTED: return "unsupported configuration";
    case FOGNET_REF_ABORTED: return "the reference run aborts (queueTime simtime overflow)";
    case FOGNET_ERR_INTERNAL: return "internal invariant check failed";
  }
  return "unknown status";
}

int fognet_create(fognet_ctx** out, int hip_device) {
  if (!out) return FOGNET_ERR_ARG;
  *out = nullptr;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) return FOGNET_ERR_DEVICE;
  if (hip_device < 0 || hip_device >= n) return FOGNET_ERR_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, hip_device) != hipSuccess) return FOGNET_ERR_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FOGNET_ERR_DEVICE;
  fognet_ctx* c = new (std::nothrow) fognet_ctx();
  if (!c) return FOGNET_ERR_OOM;
  c->device = hip_device;
  if (prop.multiProcessorCount > 0) c->cus = prop.multiProcessorCount;
  if (hipSetDevice(hip_device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return FOGNET_ERR_DEVICE;
  }
  *out = c;
  return FOGNET_OK;
}

void fognet_destroy(fognet_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->ring) (void)hipFree(c->ring);
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->red) (void)hipFree(c->red);
  if (c->host_stage) (void)hipHostFree(c->host_stage);
  if (c->hier_ev) (void)hipEventSynchronize(c->hier_ev), (void)hipEventDestroy(c->hier_ev);
  if (c->hier_host) (void)hipHostFree(c->hier_host);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

int fognet_hier_path_stats(const fognet_ctx* c, int64_t* region_launches, int64_t* sequential_launches) {
  if (!c) return FOGNET_ERR_ARG;
  if (region_launches) *region_launches = c->hier_region_launches;
  if (sequential_launches) *sequential_launches = c->hier_seq_launches;
  return FOGNET_OK;
}

const char* fognet_last_error(const fognet_ctx* c) { return c ? c->err.c_str() : "null context"; }

int fognet_sync(fognet_ctx* c) {
  if (!c) return FOGNET_ERR_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  hipError_t e = hipDeviceSynchronize();
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "hipDeviceSynchronize");
}

int fognet_decide_batch_dev(fognet_ctx* c, int policy, int64_t m, int32_t n, const double* adv_busy,
                            const int32_t* adv_mips, const int32_t* req, int32_t* out_node, int32_t* out_status,
                            void* stream) {
  if (!c) return FOGNET_ERR_ARG;
  if (policy != FOGNET_POLICY_REF_V3) return fail(c, FOGNET_ERR_UNSUPPORTED, "unknown policy");
  if (m < 0) return fail(c, FOGNET_ERR_ARG, "m < 0");
  if (m > 0 && (!out_node || (n > 0 && (!adv_busy || !adv_mips || !req))))
    return fail(c, FOGNET_ERR_ARG, "null pointer");
  int rc = set_device(c);
  if (rc) return rc;
  hipError_t e = fognet::launch_decide(m, n, n, adv_busy, adv_mips, req, out_node, out_status, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "decide launch");
}

int fognet_decide(fognet_ctx* c, int policy, int32_t n, const double* adv_busy, const int32_t* adv_mips,
                  int32_t req_mips, int32_t* out_node) {
  if (!c || !out_node) return FOGNET_ERR_ARG;
  if (policy != FOGNET_POLICY_REF_V3) return fail(c, FOGNET_ERR_UNSUPPORTED, "fognet_decide: policy REF_V3 only");
  if (n <= 0) return fail(c, FOGNET_ERR_NO_NODES, "n <= 0 (BrokerBaseApp3.cc:268 reads brokers[0])");
  if (!adv_busy || !adv_mips) return fail(c, FOGNET_ERR_ARG, "null view");
  int rc = set_device(c);
  if (rc) return rc;
  // result words at the stage's start; a view too large for the kernel arguments follows them and is
  // moved to device scratch by one DMA copy (the kernel would read it over the link at one wave's pace)
  const size_t far = n > fognet::kDecideArgNodes ? (size_t)n * sizeof(double) : 0;
  rc = ensure_host(c, 256 + far);
  if (rc) return rc;
  if (far) {
    rc = ensure(c, &c->scratch, &c->scratch_bytes, far, "decide scratch");
    if (rc) return rc;
  }
  fognet::DecideArgs a;
  a.n = n;
  a.mips0 = adv_mips[0];  // the policy reads brokers[0]->getMips() only (BrokerBaseApp3.cc:268,273)
  a.req = req_mips;
  a.pad = 0;
  unsigned char* const h = static_cast<unsigned char*>(c->host_stage);
  unsigned char* const d = static_cast<unsigned char*>(c->host_stage_dev);
  if (far) memcpy(h + 256, adv_busy, far);
  else memcpy(a.busy, adv_busy, (size_t)n * sizeof(double));
  volatile int32_t* res = reinterpret_cast<volatile int32_t*>(h);
  res[0] = -1;
  res[1] = FOGNET_ERR_DEVICE;
  hipError_t e = hipSuccess;
  if (far && (e = hipMemcpyAsync(c->scratch, h + 256, far, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return hip_fail(c, e, "decide copy-in");
  e = fognet::launch_decide_args(a, static_cast<const double*>(c->scratch), reinterpret_cast<int32_t*>(d), c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "decide launch");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "decide sync");
  if (res[1] != FOGNET_OK) return fail(c, res[1], fognet_status_string(res[1]));
  *out_node = res[0];
  return FOGNET_OK;
}

int fognet_decide_window(fognet_ctx* c, int policy, int32_t n, const double* adv_busy, const int32_t* adv_mips,
                         int32_t m, const int32_t* req_mips, int32_t* out_node) {
  if (!c || m < 0 || (m > 0 && (!out_node || !req_mips))) return fail(c, FOGNET_ERR_ARG, "decide_window: bad argument");
  if (policy != FOGNET_POLICY_REF_V3) return fail(c, FOGNET_ERR_UNSUPPORTED, "decide_window: policy REF_V3 only");
  if (m == 0) return FOGNET_OK;
  if (n <= 0) return fail(c, FOGNET_ERR_NO_NODES, "n <= 0 (BrokerBaseApp3.cc:268 reads brokers[0])");
  if (!adv_busy || !adv_mips) return fail(c, FOGNET_ERR_ARG, "null view");
  int rc = set_device(c);
  if (rc) return rc;
  // stage: [node m][status m][mips0][req m][busy n], 256-B aligned parts
  const size_t o_st = align256((size_t)m * 4), o_m0 = o_st + align256((size_t)m * 4), o_rq = o_m0 + 256;
  const size_t o_b = o_rq + align256((size_t)m * 4), total = o_b + (size_t)n * sizeof(double);
  rc = ensure_host(c, total);
  if (rc) return rc;
  unsigned char* const h = static_cast<unsigned char*>(c->host_stage);
  unsigned char* const d = static_cast<unsigned char*>(c->host_stage_dev);
  memcpy(h + o_m0, adv_mips, sizeof(int32_t));
  memcpy(h + o_rq, req_mips, (size_t)m * 4);
  memcpy(h + o_b, adv_busy, (size_t)n * sizeof(double));
  const double* view = reinterpret_cast<const double*>(d + o_b);  // small views: read in place over the link
  hipError_t e = hipSuccess;
  if (n > fognet::kDecideArgNodes) {
    rc = ensure(c, &c->scratch, &c->scratch_bytes, (size_t)n * sizeof(double), "decide scratch");
    if (rc) return rc;
    if ((e = hipMemcpyAsync(c->scratch, h + o_b, (size_t)n * sizeof(double), hipMemcpyHostToDevice, c->stream)) !=
        hipSuccess)
      return hip_fail(c, e, "decide_window copy-in");
    view = static_cast<const double*>(c->scratch);
  }
  e = fognet::launch_decide(m, n, 0, view,
                                       reinterpret_cast<const int32_t*>(d + o_m0), reinterpret_cast<const int32_t*>(d + o_rq),
                                       reinterpret_cast<int32_t*>(d), reinterpret_cast<int32_t*>(d + o_st), c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "decide_window launch");
  if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return hip_fail(c, e, "decide_window sync");
  memcpy(out_node, h, (size_t)m * 4);
  const int32_t* st = reinterpret_cast<const int32_t*>(h + o_st);
  for (int32_t i = 0; i < m; ++i)
    if (st[i] != FOGNET_OK) {
      char buf[96];
      snprintf(buf, sizeof buf, "request %d: %s", i, fognet_status_string(st[i]));
      return fail(c, st[i], buf);
    }
  return FOGNET_OK;
}

int fognet_decide_v2_batch_dev(fognet_ctx* c, int64_t m, int32_t n, const int32_t* adv_mips, const int32_t* local_mips,
                               const int32_t* req, int32_t* out_node, int32_t* out_action, void* stream) {
  if (!c) return FOGNET_ERR_ARG;
  if (m < 0 || n < 0) return fail(c, FOGNET_ERR_ARG, "m < 0 or n < 0");
  if (m > 0 && (!out_node || !out_action || !local_mips || !req || (n > 0 && !adv_mips)))
    return fail(c, FOGNET_ERR_ARG, "null pointer");
  int rc = set_device(c);
  if (rc) return rc;
  hipError_t e = fognet::launch_decide_v2(m, n, adv_mips, local_mips, req, out_node, out_action, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "decide_v2 launch");
}

int fognet_decide_v2(fognet_ctx* c, int32_t n, const int32_t* adv_mips, int32_t local_mips, int32_t req_mips,
                     int32_t* out_node, int32_t* out_action) {
  if (!c || !out_node || !out_action) return FOGNET_ERR_ARG;
  if (n < 0) return fail(c, FOGNET_ERR_ARG, "n < 0");
  if (n > 0 && !adv_mips) return fail(c, FOGNET_ERR_ARG, "null view");
  int rc = set_device(c);
  if (rc) return rc;
  const size_t nm = (size_t)n * sizeof(int32_t);
  const size_t off_s = (nm + 255) & ~(size_t)255, off_o = off_s + 256, total = off_o + 256;
  rc = ensure(c, &c->scratch, &c->scratch_bytes, total, "decide scratch");
  if (rc) return rc;
  char* s = (char*)c->scratch;
  const int32_t scal[2] = {local_mips, req_mips};
  hipError_t e;
  if ((n > 0 && (e = hipMemcpyAsync(s, adv_mips, nm, hipMemcpyHostToDevice, c->stream)) != hipSuccess) ||
      (e = hipMemcpyAsync(s + off_s, scal, sizeof scal, hipMemcpyHostToDevice, c->stream)) != hipSuccess)
    return hip_fail(c, e, "decide_v2 copy-in");
  e = fognet::launch_decide_v2(1, n, (const int32_t*)s, (const int32_t*)(s + off_s), (const int32_t*)(s + off_s) + 1,
                               (int32_t*)(s + off_o), (int32_t*)(s + off_o) + 1, c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "decide_v2 launch");
  int32_t res[2] = {-1, 0};
  if ((e = hipMemcpyAsync(res, s + off_o, sizeof res, hipMemcpyDeviceToHost, c->stream)) != hipSuccess ||
      (e = hipStreamSynchronize(c->stream)) != hipSuccess)
    return hip_fail(c, e, "decide_v2 copy-out");
  *out_node = res[0];
  *out_action = res[1];
  return FOGNET_OK;
}

static int stage(fognet_ctx* c, const fognet_batch_in* in, fognet_batch_out* out, void* stream, int which) {
  if (!c || !out) return FOGNET_ERR_ARG;
  fognet::ReplayArgs a;
  int rc = prepare(c, in, &a);
  if (rc) return rc;
  if (!out->stats) return fail(c, FOGNET_ERR_ARG, "stats output is required (per-replication status)");
  const int n_null = !out->node + !out->status + !out->start_tick + !out->done_tick;
  if (n_null != 0 && n_null != 4)
    return fail(c, FOGNET_ERR_ARG, "per-task outputs: give all four arrays, or none (statistics only)");
  const bool stats_only = n_null == 4 && a.T > 0;
  if (stats_only && which != 3)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "statistics-only replays run through fognet_run_batch_dev");
  if (a.R == 0) return FOGNET_OK;
  rc = set_device(c);
  if (rc) return rc;
  a.out_node = out->node;
  a.out_status = out->status;
  a.out_start = out->start_tick;
  a.out_done = out->done_tick;
  a.out_stats = out->stats;
  a.out_energy = out->node_energy_j;
  a.hist = out->hist;
  if (a.out_energy && !a.p_busy) return fail(c, FOGNET_ERR_ARG, "node_energy_j needs the power model (p_busy_w/p_idle_w)");
  hipError_t e = hipSuccess;
  if (use_wide(a.N) || a.down || a.policy == FOGNET_POLICY_EXT_HIER) {  // (regions: the wide kernel's groups)
    // crashes are only modelled by the wide kernel; it accumulates the statistics while it replays, so the
    // statistics-only stage has nothing left to do
    if (!(which & 1)) return FOGNET_OK;
    a.no_task_out = stats_only ? 1 : 0;
    const int32_t B = (a.N + FOGNET_HIER_REGION_NODES - 1) / FOGNET_HIER_REGION_NODES;
    const bool hier_split = a.policy == FOGNET_POLICY_EXT_HIER && !a.down && !stats_only && a.T > 0 && B >= 2;
    bool regions = hier_split && use_regions();
    // resume (replay_region.hip): an escalated replication continues on the sequential kernel from
    // its first escalated publish, so the region pass is never wasted and is always taken
    const bool resume = regions && use_resume();
    const fognet_ctx::HierShape shape{a.R, a.T, a.N, stream};
    if (regions && regions_auto() && !resume) {
      // the last region pass's hand-over count, if it has reached the host (never waited for)
      if (c->hier_pending && hipEventQuery(c->hier_ev) == hipSuccess) {
        c->hier_pending = false;
        c->hier_seq = 2 * (int64_t)c->hier_host[0] > (int64_t)c->hier_pend_shape.R;
        c->hier_seq_shape = c->hier_pend_shape;
        c->hier_seq_runs = 0;
      }
      if (c->hier_seq && !(c->hier_seq_shape == shape)) c->hier_seq = false;  // another job: measure it
      if (c->hier_seq && c->hier_seq_runs < kHierReprobe) {
        regions = false;  // most replications escalated: the region pass would only be replayed again
        ++c->hier_seq_runs;
      } else {
        c->hier_seq = false;  // (measure again)
      }
    }
    if (hier_split) ++(regions ? c->hier_region_launches : c->hier_seq_launches);
    if (regions) {
      // one wavefront per (replication, region) while no region escalates (replay_region.hip), the
      // statistics pass, then the sequential wide kernel for the replications some region handed back.
      // workspace: [hand-over counter | list [R] | first escalations [R] | region records [R][B] | segment
      // offsets [R][B+1] | dispatch keys [R][B] | dispatch order [R*B] | resume records [R] | node tails
      // [R][N][2] | entries [R][T] | node records [R][N] | busy view [R][B][1024] | region-sorted trace and
      // outputs [R][T] | sorted -> trace index [R][T]] + the hand-over launch's space, after it (resume: the
      // wide kernel reads the region state), else from the entries on (stream order: after the finish
      // kernel has read the node records and the sorted outputs), with one workspace slot per handed-over
      // replication up to kWideFallbackSlots (an escalation-heavy job replays its hand-overs side by side,
      // as the sequential-only path does)
      const size_t RT = (size_t)a.R * (size_t)a.T;
      const size_t o_esc = align256(256 + (size_t)a.R * sizeof(int32_t));
      const size_t o_rec = o_esc + align256((size_t)a.R * sizeof(int32_t));
      const size_t o_seg = o_rec + align256((size_t)a.R * (size_t)B * sizeof(fognet::RegionRec));
      const size_t o_ok = o_seg + align256((size_t)a.R * (size_t)(B + 1) * sizeof(int32_t));
      const size_t o_perm = o_ok + align256((size_t)a.R * (size_t)B * sizeof(uint32_t));
      const size_t o_pacc = o_perm + align256((size_t)a.R * (size_t)B * sizeof(int32_t));
      const size_t o_tails = o_pacc + align256((size_t)a.R * fognet::kRegionResumeBytes);
      const size_t o_e = o_tails + align256((size_t)a.R * (size_t)a.N * 2 * sizeof(int64_t));
      const size_t o_nd = o_e + align256(RT * sizeof(fognet::WideEntry));
      const size_t o_vb = o_nd + align256((size_t)a.R * (size_t)a.N * sizeof(fognet::WideNode));
      const size_t o_sa = o_vb + align256((size_t)a.R * (size_t)B * FOGNET_HIER_REGION_NODES * sizeof(uint32_t));
      const size_t o_sq = o_sa + align256(RT * sizeof(int64_t));
      const size_t o_inv = o_sq + align256(RT * sizeof(int32_t));
      const size_t o_on = o_inv + align256(RT * sizeof(int32_t));
      const size_t o_os = o_on + align256(RT * sizeof(int32_t));
      const size_t o_ost = o_os + align256(RT);
      const size_t o_od = o_ost + align256(RT * sizeof(int64_t));
      const size_t o_sidx = o_od + align256(RT * sizeof(int64_t));
      const size_t body = o_sidx + align256(RT * sizeof(int32_t)) - o_e;
      const int32_t slots = a.R < kWideFallbackSlots ? a.R : kWideFallbackSlots;
      const size_t fb = fognet::replay_wide_workspace_bytes(slots, a.T, a.N, false, a.policy);
      const size_t o_wide = resume ? o_e + body : o_e;
      const size_t total = resume ? o_wide + fb : o_e + (body > fb ? body : fb);
      rc = ensure(c, (void**)&c->ring, &c->ring_bytes, total, "region replay workspace");
      if (rc) return rc;
      unsigned char* const base = reinterpret_cast<unsigned char*>(c->ring);
      a.wide_count = reinterpret_cast<int32_t*>(base);
      a.wide_list = reinterpret_cast<int32_t*>(base + 256);
      e = hipMemsetAsync(a.wide_count, 0, sizeof(int32_t), (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(c, e, "hand-over counter");
      fognet::RegionWs w;
      w.e = reinterpret_cast<fognet::WideEntry*>(base + o_e);
      w.nd = reinterpret_cast<fognet::WideNode*>(base + o_nd);
      w.rec = reinterpret_cast<fognet::RegionRec*>(base + o_rec);
      w.vb = reinterpret_cast<uint32_t*>(base + o_vb);
      w.esc = reinterpret_cast<int32_t*>(base + o_esc);  // (set by the sort kernel)
      w.s_idx = reinterpret_cast<int32_t*>(base + o_sidx);
      w.pacc = base + o_pacc;
      w.pass = 1;
      w.seg = reinterpret_cast<int32_t*>(base + o_seg);
      w.okey = reinterpret_cast<uint32_t*>(base + o_ok);
      w.perm = reinterpret_cast<int32_t*>(base + o_perm);
      w.tails = reinterpret_cast<int64_t*>(base + o_tails);
      w.s_arr = reinterpret_cast<int64_t*>(base + o_sa);
      w.s_req = reinterpret_cast<int32_t*>(base + o_sq);
      w.inv = reinterpret_cast<int32_t*>(base + o_inv);
      w.o_node = reinterpret_cast<int32_t*>(base + o_on);
      w.o_status = reinterpret_cast<uint8_t*>(base + o_os);
      w.o_start = reinterpret_cast<int64_t*>(base + o_ost);
      w.o_done = reinterpret_cast<int64_t*>(base + o_od);
      w.B = B;
      if (regions_only()) a.wide_list = nullptr;
      e = fognet::launch_replay_region(a, w, resume && !regions_only(), (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(c, e, "region replay launch");
      if (regions_only()) return FOGNET_OK;
      e = fognet::launch_replay_wide(a, base + o_wide, slots, (hipStream_t)stream, resume ? &w : nullptr);
      if (e != hipSuccess) return hip_fail(c, e, "wide hand-over launch");
      if (regions_auto() && !resume && !c->hier_pending) {  // the hand-over count back to the host, asynchronously
        // (while a measurement is in flight, later launches are not measured: its pinned slot and event
        // stay paired with the launch that issued them)
        if (!c->hier_host && hipHostMalloc((void**)&c->hier_host, sizeof(int32_t), hipHostMallocDefault) != hipSuccess)
          c->hier_host = nullptr;
        if (!c->hier_ev && hipEventCreateWithFlags(&c->hier_ev, hipEventDisableTiming) != hipSuccess) c->hier_ev = nullptr;
        if (c->hier_host && c->hier_ev) {
          c->hier_pend_shape = shape;
          e = hipMemcpyAsync(c->hier_host, a.wide_count, sizeof(int32_t), hipMemcpyDeviceToHost, (hipStream_t)stream);
          if (e == hipSuccess) e = hipEventRecord(c->hier_ev, (hipStream_t)stream);
          if (e != hipSuccess) return hip_fail(c, e, "hand-over count copy");
          c->hier_pending = true;
        }
      }
      return FOGNET_OK;
    }
    const size_t ws = fognet::replay_wide_workspace_bytes(a.R, a.T, a.N, false, a.policy);
    rc = ensure(c, (void**)&c->ring, &c->ring_bytes, ws, "wide replay workspace");
    if (rc) return rc;
    e = fognet::launch_replay_wide(a, c->ring, a.R, (hipStream_t)stream);
    return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "wide replay launch");
  }
  // both stages: the replay kernel runs the statistics pass as its epilogue
  a.fuse_stats = which == 3 ? 1 : 0;
  if (a.fuse_stats) which = 1;
  // statistics accumulated in the loop (replay_inl_kernel) where the node tails hold exact totals
  a.inloop = a.fuse_stats && (uint64_t)a.T * (uint64_t)a.max_s < (1ull << 32) && use_inloop() ? 1 : 0;
  if (a.inloop) a.no_task_out = stats_only ? 1 : 0;
  if (which & 1) {
    // workspace: [hand-over counter | hand-over list [R] | pending-task rings, reused by the wide kernel's
    // replay of the handed-over replications once the register kernel is done (stream order)]
    // + for a statistics-only replay the per-task outputs the fused statistics epilogue reads back
    const size_t ring_bytes = (size_t)a.R * (size_t)a.N * ((size_t)1 << a.q_log2) * sizeof(fognet::RingWord);
    const int32_t slots = fallback_slots(a.R, a.T, a.N, ring_bytes, false, a.policy);
    const size_t fb_bytes = fognet::replay_wide_workspace_bytes(slots, a.T, a.N, false, a.policy);
    const size_t o_board = align256(256 + (size_t)a.R * sizeof(int32_t));
    const size_t head = o_board + fognet::kBoardWords * sizeof(uint32_t);
    const size_t body = ring_bytes > fb_bytes ? ring_bytes : fb_bytes;
    const size_t RT = stats_only && !a.inloop ? (size_t)a.R * (size_t)a.T : 0;
    const size_t o_node = head + align256(body), o_st = o_node + align256(RT * 4), o_start = o_st + align256(RT),
                 o_done = o_start + align256(RT * 8), total = o_done + align256(RT * 8);
    rc = ensure(c, (void**)&c->ring, &c->ring_bytes, total, "ring workspace");
    if (rc) return rc;
    unsigned char* const base = reinterpret_cast<unsigned char*>(c->ring);
    a.wide_count = reinterpret_cast<int32_t*>(base);
    a.wide_list = reinterpret_cast<int32_t*>(base + 256);
    a.ring = reinterpret_cast<fognet::RingWord*>(base + head);
    if (stats_only && !a.inloop) {
      a.out_node = reinterpret_cast<int32_t*>(base + o_node);
      a.out_status = reinterpret_cast<uint8_t*>(base + o_st);
      a.out_start = reinterpret_cast<int64_t*>(base + o_start);
      a.out_done = reinterpret_cast<int64_t*>(base + o_done);
    }
    e = hipMemsetAsync(a.wide_count, 0, sizeof(int32_t), (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "hand-over counter");
    if (!a.inloop) {  // replay_kernel's progress board: every slot empty
      a.board = reinterpret_cast<uint32_t*>(base + o_board);
      e = hipMemsetAsync(a.board, 0xFF, fognet::kBoardWords * sizeof(uint32_t), (hipStream_t)stream);
      if (e != hipSuccess) return hip_fail(c, e, "progress board");
    }
    e = fognet::launch_replay(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "replay launch");
    // the handed-over replications (usually none: every workgroup leaves at once).  The wide kernel
    // accumulates its statistics inline; in a replay-only call the statistics stage that follows
    // recomputes them for every replication from the per-task outputs, so the hand-over must not add
    // its histogram and energy as well
    fognet::ReplayArgs hw = a;
    if (!a.fuse_stats) {
      hw.hist = nullptr;
      hw.out_energy = nullptr;
    }
    e = fognet::launch_replay_wide(hw, base + head, slots, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "wide hand-over launch");
  }
  if (which & 2) {
    e = fognet::launch_rep_stats(a, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(c, e, "stats launch");
  }
  return FOGNET_OK;
}

int fognet_run_generated_dev(fognet_ctx* c, const fognet_gen_params* p, int64_t r0, const fognet_batch_in* in,
                             fognet_batch_out* out, void* stream) {
  if (!c || !p || !in || !out) return FOGNET_ERR_ARG;
  if (in->arrive_tick || in->req_mips || in->mips || in->dl_tick || in->ul_tick || in->init_adv_tick || in->down_tick ||
      in->region)
    return fail(c, FOGNET_ERR_ARG, "generated replay: the trace and node-parameter arrays must be NULL (generated)");
  // (EXT_HIER: each publish's region from the mobility model of fa.mobility_regions, computed in the
  // kernel, replication by replication on the sequential wide kernel)
  if (out->node || out->status || out->start_tick || out->done_tick)
    return fail(c, FOGNET_ERR_ARG, "generated replay: statistics only (per-task arrays must be NULL)");
  if (!out->stats) return fail(c, FOGNET_ERR_ARG, "stats output is required (per-replication status)");
  if (r0 < 0 || p->req_lo < 0 || p->req_hi < p->req_lo) return fail(c, FOGNET_ERR_ARG, "bad r0 or req range");
  if (in->R > 0 && (!p->mean_gap_ticks || !p->lat_scale)) return fail(c, FOGNET_ERR_ARG, "null generator parameters");
  // the register kernel's in-loop statistics take per-node totals from the node tails' 32-bit
  // cumulative service (MIPS >= 1000): past 2^32 service seconds per replication the wide kernel
  // (64-bit cumulative sums) replays the generated traces instead
  const bool long_run = in->T > 0 && (uint64_t)in->T * (uint64_t)(p->req_hi / 1000) >= (1ull << 32);
  fognet::ReplayArgs a;
  int rc = prepare(c, in, &a, true);
  if (rc) return rc;
  if (a.R == 0) return FOGNET_OK;
  rc = set_device(c);
  if (rc) return rc;
  a.gen_on = 1;
  a.gen_r0 = r0;
  a.gen = *p;
  a.no_task_out = 1;
  a.out_stats = out->stats;
  a.out_energy = out->node_energy_j;
  a.hist = out->hist;
  if (a.out_energy && !a.p_busy) return fail(c, FOGNET_ERR_ARG, "node_energy_j needs the power model (p_busy_w/p_idle_w)");
  hipError_t e;
  if (use_wide(a.N) || long_run || a.policy == FOGNET_POLICY_EXT_HIER) {
    const size_t ws = fognet::replay_wide_workspace_bytes(a.R, a.T, a.N, true, a.policy);
    rc = ensure(c, (void**)&c->ring, &c->ring_bytes, ws, "wide replay workspace");
    if (rc) return rc;
    e = fognet::launch_replay_wide(a, c->ring, a.R, (hipStream_t)stream);
    return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "wide replay launch");
  }
  // workspace: [hand-over counter, work counter | list [R] | rings of the resident workgroups, reused by
  // the wide hand-over]
  const int64_t resident = (int64_t)c->cus * fognet::kGenWavesPerCu;
  a.gen_slots = (int32_t)(a.R < resident ? a.R : resident);
  const size_t ring_bytes = (size_t)a.gen_slots * (size_t)a.N * ((size_t)1 << a.q_log2) * sizeof(fognet::RingWord);
  const int32_t slots = fallback_slots(a.R, a.T, a.N, ring_bytes, true, a.policy);
  const size_t fb_bytes = fognet::replay_wide_workspace_bytes(slots, a.T, a.N, true, a.policy);
  const size_t head = align256(256 + (size_t)a.R * sizeof(int32_t));
  rc = ensure(c, (void**)&c->ring, &c->ring_bytes, head + (ring_bytes > fb_bytes ? ring_bytes : fb_bytes),
              "ring workspace");
  if (rc) return rc;
  unsigned char* const base = reinterpret_cast<unsigned char*>(c->ring);
  a.wide_count = reinterpret_cast<int32_t*>(base);
  a.wide_list = reinterpret_cast<int32_t*>(base + 256);
  a.ring = reinterpret_cast<fognet::RingWord*>(base + head);
  a.queue = reinterpret_cast<int32_t*>(base + sizeof(int32_t));
  e = hipMemsetAsync(base, 0, 2 * sizeof(int32_t), (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "hand-over and work counters");
  e = fognet::launch_replay(a, (hipStream_t)stream);
  if (e != hipSuccess) return hip_fail(c, e, "replay launch");
  e = fognet::launch_replay_wide(a, base + head, slots, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "wide hand-over launch");
}

int fognet_replay_dev(fognet_ctx* c, const fognet_batch_in* in, fognet_batch_out* out, void* stream) {
  return stage(c, in, out, stream, 1);
}

int fognet_rep_stats_dev(fognet_ctx* c, const fognet_batch_in* in, fognet_batch_out* out, void* stream) {
  return stage(c, in, out, stream, 2);
}

int fognet_run_batch_dev(fognet_ctx* c, const fognet_batch_in* in, fognet_batch_out* out, void* stream) {
  return stage(c, in, out, stream, 3);
}

int fognet_run_batch(fognet_ctx* c, const fognet_batch_in* in, fognet_batch_out* out) {
  if (!c || !in || !out) return FOGNET_ERR_ARG;
  fognet::ReplayArgs chk;
  int rc = prepare(c, in, &chk);
  if (rc) return rc;
  rc = set_device(c);
  if (rc) return rc;
  const size_t R = (size_t)in->R, T = (size_t)in->T, N = (size_t)in->N;
  const size_t NR = in->node_stride ? R : 1;
  const size_t HB = FOGNET_HIST_METRICS * FOGNET_HIST_BINS * sizeof(int64_t);
  const bool pw = in->p_busy_w != nullptr;
  const bool dn = in->down_tick != nullptr;
  // inputs 0..8, outputs 9..15, region 16
  const void* hsrc[9] = {in->arrive_tick, in->req_mips, in->mips, in->dl_tick, in->ul_tick, in->init_adv_tick,
                         in->p_busy_w, in->p_idle_w, in->down_tick};
  const size_t isz[9] = {R * T * 8, R * T * 4, NR * N * 4, NR * N * 8, NR * N * 8, NR * N * 8,
                         pw ? NR * N * 8 : 0, pw ? NR * N * 8 : 0, dn ? NR * N * 8 : 0};
  const bool rg = in->policy == FOGNET_POLICY_EXT_HIER && in->region != nullptr;
  void* hdst[7] = {out->node, out->status, out->start_tick, out->done_tick, out->stats, out->node_energy_j,
                   out->hist};
  const size_t osz[7] = {R * T * 4, R * T * 1, R * T * 8, R * T * 8, R * sizeof(fognet_rep_stats),
                         out->node_energy_j ? R * N * 8 : 0, out->hist ? HB : 0};
  void* d[17] = {};
  auto cleanup = [&]() {
    for (int i = 0; i < 17; ++i)
      if (d[i]) (void)hipFree(d[i]);
  };
  if (rg) {
    hipError_t e = hipMalloc(&d[16], R * T * 4 ? R * T * 4 : 8);
    if (e == hipSuccess && R * T) e = hipMemcpyAsync(d[16], in->region, R * T * 4, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(c, e, "region copy-in");
    }
  }
  for (int i = 0; i < 16; ++i) {
    const size_t sz = i < 9 ? isz[i] : osz[i - 9];
    if (i >= 6 && i < 8 && !pw) continue;
    if (i == 8 && !dn) continue;
    if (i >= 9 && i < 13 && !hdst[i - 9]) continue;  // statistics only: no per-task outputs
    if (i >= 14 && !hdst[i - 9]) continue;
    hipError_t e = hipMalloc(&d[i], sz ? sz : 8);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(c, e, "hipMalloc batch");
    }
    if (i < 9 && sz) e = hipMemcpyAsync(d[i], hsrc[i], sz, hipMemcpyHostToDevice, c->stream);
    if (i == 15 && e == hipSuccess) e = hipMemcpyAsync(d[i], hdst[6], sz, hipMemcpyHostToDevice, c->stream);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(c, e, "copy-in");
    }
  }
  fognet_batch_in din = *in;
  din.arrive_tick = (const int64_t*)d[0];
  din.req_mips = (const int32_t*)d[1];
  din.mips = (const int32_t*)d[2];
  din.dl_tick = (const int64_t*)d[3];
  din.ul_tick = (const int64_t*)d[4];
  din.init_adv_tick = (const int64_t*)d[5];
  din.p_busy_w = (const double*)d[6];
  din.p_idle_w = (const double*)d[7];
  din.down_tick = (const int64_t*)d[8];
  din.region = (const int32_t*)d[16];
  fognet_batch_out dout = {(int32_t*)d[9], (uint8_t*)d[10], (int64_t*)d[11], (int64_t*)d[12],
                           (fognet_rep_stats*)d[13], (double*)d[14], (int64_t*)d[15]};
  rc = fognet_run_batch_dev(c, &din, &dout, c->stream);
  if (rc) {
    cleanup();
    return rc;
  }
  for (int i = 0; i < 7; ++i) {
    if (!hdst[i] || !osz[i]) continue;
    hipError_t e = hipMemcpyAsync(hdst[i], d[9 + i], osz[i], hipMemcpyDeviceToHost, c->stream);
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(c, e, "copy-out");
    }
  }
  hipError_t e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    cleanup();
    return hip_fail(c, e, "batch sync");
  }
  cleanup();
  if (out->stats)
    for (size_t r = 0; r < R; ++r)
      if (out->stats[r].status != FOGNET_OK) {
        char buf[96];
        snprintf(buf, sizeof buf, "replication %zu: %s", r, fognet_status_string(out->stats[r].status));
        return fail(c, out->stats[r].status, buf);
      }
  return FOGNET_OK;
}

int fognet_user_stats_dev(fognet_ctx* c, const fognet_batch_in* in, const fognet_batch_out* out, const int64_t* user_ul,
                          const int64_t* user_dl, int32_t user_per_task, fognet_user_stats* user_stats, void* stream) {
  if (!c || !out) return FOGNET_ERR_ARG;
  fognet::ReplayArgs a;
  int rc = prepare(c, in, &a);
  if (rc) return rc;
  if (user_per_task != 0 && user_per_task != 1) return fail(c, FOGNET_ERR_ARG, "user_per_task must be 0 or 1");
  if (a.R == 0) return FOGNET_OK;
  if (!user_ul || !user_dl || !user_stats || !out->stats || (a.T > 0 && (!out->node || !out->status || !out->done_tick)))
    return fail(c, FOGNET_ERR_ARG, "null pointer");
  rc = set_device(c);
  if (rc) return rc;
  a.out_node = out->node;
  a.out_status = out->status;
  a.out_done = out->done_tick;
  a.out_stats = out->stats;
  hipError_t e = fognet::launch_user_stats(a, user_ul, user_dl, user_per_task, user_stats, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "user stats launch");
}

int fognet_run_v2_dev(fognet_ctx* c, const fognet_v2_in* in, fognet_v2_out* out, void* stream) {
  if (!c || !in || !out) return FOGNET_ERR_ARG;
  if (in->R < 0 || in->T < 0 || in->N < 0) return fail(c, FOGNET_ERR_ARG, "negative R/T/N");
  if (in->N > FOGNET_V2_MAX_NODES)
    return fail(c, FOGNET_ERR_UNSUPPORTED, "the v2 replay keeps at most 256 nodes per lane: N <= 16384");
  if (in->node_stride != 0 && in->node_stride != in->N) return fail(c, FOGNET_ERR_ARG, "node_stride must be 0 or N");
  const int q = in->queue_capacity ? in->queue_capacity : 256;
  if (q < 2 || (q & (q - 1)) != 0 || q > (1 << 16)) return fail(c, FOGNET_ERR_ARG, "queue_capacity must be a power of two in [2, 2^16]");
  int qlog = 0;
  while ((1 << qlog) < q) ++qlog;
  if (in->R == 0) return FOGNET_OK;
  if (!in->broker_mips || !in->required_time_s || !in->stop_tick || (in->T > 0 && (!in->arrive_tick || !in->req_mips)) ||
      (in->N > 0 && (!in->mips || !in->dl_tick || !in->ul_tick || !in->first_adv_tick)))
    return fail(c, FOGNET_ERR_ARG, "null input array");
  if (!out->stats || (in->T > 0 && (!out->node || !out->status || !out->start_tick || !out->done_tick)))
    return fail(c, FOGNET_ERR_ARG, "null output array");
  int rc = set_device(c);
  if (rc) return rc;
  rc = ensure(c, (void**)&c->ring, &c->ring_bytes, fognet::replay_v2_workspace_bytes(in->R, in->T, in->N, qlog),
              "v2 replay workspace");
  if (rc) return rc;
  hipError_t e = fognet::launch_replay_v2(*in, *out, c->ring, qlog, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "v2 replay launch");
}

int fognet_reduce_stats_dev(fognet_ctx* c, const fognet_rep_stats* stats, int32_t R, fognet_job_stats* out,
                            void* stream) {
  if (!c || !out || (R > 0 && !stats) || R < 0) return FOGNET_ERR_ARG;
  int rc = set_device(c);
  if (rc) return rc;
  const int32_t np = fognet::reduce_stats_parts(R);
  if (np > 0) {
    rc = ensure(c, &c->red, &c->red_bytes, (size_t)np * sizeof(fognet_job_stats), "reduction partials");
    if (rc) return rc;
  }
  hipError_t e = fognet::launch_reduce_stats(stats, R, out, static_cast<fognet_job_stats*>(c->red),
                                             (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "reduce launch");
}

void fognet_job_stats_init(fognet_job_stats* s) {
  if (!s) return;
  memset(s, 0, sizeof *s);
  s->queue_min_raw = s->resp_min_ticks = INT64_MAX;
  s->queue_max_raw = s->resp_max_ticks = s->last_tick = INT64_MIN;
}

static void add192_host(uint64_t* a, const uint64_t* b) {
  unsigned __int128 s = (unsigned __int128)a[0] + b[0];
  a[0] = (uint64_t)s;
  s = (unsigned __int128)a[1] + b[1] + (uint64_t)(s >> 64);
  a[1] = (uint64_t)s;
  a[2] = a[2] + b[2] + (uint64_t)(s >> 64);
}

void fognet_job_stats_merge(fognet_job_stats* a, const fognet_job_stats* b) {
  if (!a || !b) return;
  a->n_reps += b->n_reps;
  a->n_failed += b->n_failed;
  a->n_tasks += b->n_tasks;
  a->n_queued += b->n_queued;
  a->n_started += b->n_started;
  a->events += b->events;
  if (b->last_tick > a->last_tick) a->last_tick = b->last_tick;
  if (b->queue_min_raw < a->queue_min_raw) a->queue_min_raw = b->queue_min_raw;
  if (b->queue_max_raw > a->queue_max_raw) a->queue_max_raw = b->queue_max_raw;
  a->n_qtime += b->n_qtime;
  a->n_qtime_overflow += b->n_qtime_overflow;
  a->n_ref_aborted += b->n_ref_aborted;
  if (b->resp_min_ticks < a->resp_min_ticks) a->resp_min_ticks = b->resp_min_ticks;
  if (b->resp_max_ticks > a->resp_max_ticks) a->resp_max_ticks = b->resp_max_ticks;
  if (b->max_pending > a->max_pending) a->max_pending = b->max_pending;
  a->busy_s += b->busy_s;
  a->energy_j = a->energy_j + b->energy_j;
  add192_host(a->queue_sum, b->queue_sum);
  add192_host(a->queue_sq, b->queue_sq);
  add192_host(a->resp_sum, b->resp_sum);
  add192_host(a->resp_sq, b->resp_sq);
}

void fognet_job_stats_add_rep(fognet_job_stats* a, const fognet_rep_stats* s) {
  if (!a || !s) return;
  a->n_reps += 1;
  /* counted under FOGNET_FLAG_REF_ABORT too (status FOGNET_REF_ABORTED), like reduce_kernel */
  if ((s->status == FOGNET_OK || s->status == FOGNET_REF_ABORTED) && s->abort_tick != INT64_MAX) a->n_ref_aborted += 1;
  if (s->status != FOGNET_OK) {
    a->n_failed += 1;
    return;
  }
  fognet_job_stats b;
  fognet_job_stats_init(&b);
  b.n_tasks = s->n_tasks;
  b.n_queued = s->n_queued;
  b.n_started = s->n_started;
  b.events = s->events;
  b.last_tick = s->last_tick;
  b.queue_min_raw = s->queue_min_raw;
  b.queue_max_raw = s->queue_max_raw;
  b.n_qtime = s->n_qtime;
  b.n_qtime_overflow = s->n_qtime_overflow;
  b.resp_min_ticks = s->resp_min_ticks;
  b.resp_max_ticks = s->resp_max_ticks;
  b.max_pending = s->max_pending;
  b.busy_s = s->busy_s;
  b.energy_j = s->energy_j;
  b.queue_sum[0] = s->queue_sum_lo;
  b.queue_sum[1] = s->queue_sum_hi;
  b.queue_sum[2] = (int64_t)s->queue_sum_hi < 0 ? ~(uint64_t)0 : 0;  // two's complement sign extension
  b.queue_sq[0] = s->queue_sq_lo;
  b.queue_sq[1] = s->queue_sq_hi;
  b.queue_sq[2] = s->queue_sq_top;
  b.resp_sum[0] = s->resp_sum_lo;
  b.resp_sum[1] = s->resp_sum_hi;
  b.resp_sq[0] = s->resp_sq_lo;
  b.resp_sq[1] = s->resp_sq_hi;
  fognet_job_stats_merge(a, &b);
}

int fognet_gen_trace_dev(fognet_ctx* c, const fognet_gen_params* p, int64_t r0, int32_t R, int32_t T, int32_t N,
                         int64_t* arrive_tick, int32_t* req_mips, int32_t* mips, int64_t* dl_tick, int64_t* ul_tick,
                         int64_t* init_adv_tick, void* stream) {
  if (!c || !p) return FOGNET_ERR_ARG;
  if (R < 0 || T < 0 || N <= 0 || r0 < 0) return fail(c, FOGNET_ERR_ARG, "bad sizes");
  if (p->req_lo < 0 || p->req_hi < p->req_lo) return fail(c, FOGNET_ERR_ARG, "bad req range");
  if (R > 0 && (!p->mean_gap_ticks || !p->lat_scale || !mips || !dl_tick || !ul_tick || !init_adv_tick ||
                (T > 0 && (!arrive_tick || !req_mips))))
    return fail(c, FOGNET_ERR_ARG, "null pointer");
  int rc = set_device(c);
  if (rc) return rc;
  hipError_t e = fognet::launch_gen_trace(*p, r0, R, T, N, arrive_tick, req_mips, mips, dl_tick, ul_tick,
                                          init_adv_tick, (hipStream_t)stream);
  return e == hipSuccess ? FOGNET_OK : hip_fail(c, e, "tracegen launch");
}

}  // extern "C"

// ---------------------------------------------------------------- RCCL stats exchange
// RCCL's C API, resolved with dlsym on first use (no link-time dependency).
namespace {

typedef struct {
  char internal[FOGNET_COMM_ID_BYTES];
} RcclId;
typedef void* RcclComm;
enum { kRcclInt8 = 0, kRcclUint8 = 1, kRcclInt64 = 4, kRcclSum = 0 };

struct Rccl {
  int (*get_unique_id)(RcclId*) = nullptr;
  int (*comm_init_rank)(RcclComm*, int, RcclId, int) = nullptr;
  int (*comm_destroy)(RcclComm) = nullptr;
  int (*all_gather)(const void*, void*, size_t, int, RcclComm, hipStream_t) = nullptr;
  int (*all_reduce)(const void*, void*, size_t, int, int, RcclComm, hipStream_t) = nullptr;
  const char* (*error_string)(int) = nullptr;
  bool ok = false;
  std::string why;
};

Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      x.why = std::string("cannot load librccl: ") + dlerror();
      return x;
    }
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    x.all_gather = reinterpret_cast<decltype(x.all_gather)>(dlsym(h, "ncclAllGather"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.comm_init_rank && x.comm_destroy && x.all_gather && x.all_reduce && x.error_string;
    if (!x.ok) x.why = "librccl lacks the NCCL collective API";
    return x;
  }();
  return r;
}

int rccl_fail(fognet_ctx* c, int e, const char* what) {
  return fail(c, FOGNET_ERR_DEVICE, std::string(what) + ": " + rccl().error_string(e));
}

}  // namespace

struct fognet_comm {
  RcclComm comm = nullptr;
  int32_t world = 0, rank = 0;
  int device = -1;
  void* buf = nullptr;  // [world] job records
};

extern "C" {

int fognet_comm_unique_id(uint8_t id[FOGNET_COMM_ID_BYTES]) {
  if (!id) return FOGNET_ERR_ARG;
  Rccl& r = rccl();
  if (!r.ok) return FOGNET_ERR_UNSUPPORTED;
  RcclId x;
  if (r.get_unique_id(&x) != 0) return FOGNET_ERR_DEVICE;
  memcpy(id, x.internal, FOGNET_COMM_ID_BYTES);
  return FOGNET_OK;
}

int fognet_comm_create(fognet_ctx* c, int32_t world, int32_t rank, const uint8_t id[FOGNET_COMM_ID_BYTES],
                       fognet_comm** out) {
  if (!c || !out || !id || world <= 0 || rank < 0 || rank >= world) return fail(c, FOGNET_ERR_ARG, "comm: bad world/rank");
  *out = nullptr;
  Rccl& r = rccl();
  if (!r.ok) return fail(c, FOGNET_ERR_UNSUPPORTED, r.why);
  int rc = set_device(c);
  if (rc) return rc;
  fognet_comm* m = new fognet_comm;
  m->world = world;
  m->rank = rank;
  m->device = c->device;
  RcclId x;
  memcpy(x.internal, id, FOGNET_COMM_ID_BYTES);
  const int e = r.comm_init_rank(&m->comm, world, x, rank);
  if (e != 0) {
    delete m;
    return rccl_fail(c, e, "ncclCommInitRank");
  }
  const hipError_t he = hipMalloc(&m->buf, (size_t)world * sizeof(fognet_job_stats));
  if (he != hipSuccess) {
    r.comm_destroy(m->comm);
    delete m;
    return hip_fail(c, he, "hipMalloc comm buffer");
  }
  *out = m;
  return FOGNET_OK;
}

void fognet_comm_destroy(fognet_comm* m) {
  if (!m) return;
  (void)hipSetDevice(m->device);
  if (m->comm) rccl().comm_destroy(m->comm);
  if (m->buf) (void)hipFree(m->buf);
  delete m;
}

int fognet_allreduce_stats(fognet_ctx* c, fognet_comm* m, fognet_job_stats* inout, int64_t* hist, void* stream) {
  if (!c || !m || !inout) return fail(c, FOGNET_ERR_ARG, "allreduce_stats: null argument");
  if (m->device != c->device) return fail(c, FOGNET_ERR_ARG, "allreduce_stats: comm and context on different devices");
  int rc = set_device(c);
  if (rc) return rc;
  Rccl& r = rccl();
  hipStream_t s = (hipStream_t)stream;
  const size_t sz = sizeof(fognet_job_stats);
  unsigned char* const buf = static_cast<unsigned char*>(m->buf);
  hipError_t he = hipMemcpyAsync(buf + (size_t)m->rank * sz, inout, sz, hipMemcpyHostToDevice, s);
  if (he != hipSuccess) return hip_fail(c, he, "allreduce_stats copy-in");
  int e = r.all_gather(buf + (size_t)m->rank * sz, buf, sz, kRcclUint8, m->comm, s);  // in place
  if (e != 0) return rccl_fail(c, e, "ncclAllGather");
  if (hist) {
    e = r.all_reduce(hist, hist, (size_t)FOGNET_HIST_METRICS * FOGNET_HIST_BINS, kRcclInt64, kRcclSum, m->comm, s);
    if (e != 0) return rccl_fail(c, e, "ncclAllReduce");
  }
  std::string recs((size_t)m->world * sz, '\0');
  he = hipMemcpyAsync(&recs[0], buf, recs.size(), hipMemcpyDeviceToHost, s);
  if (he == hipSuccess) he = hipStreamSynchronize(s);
  if (he != hipSuccess) return hip_fail(c, he, "allreduce_stats copy-out");
  fognet_job_stats acc;
  fognet_job_stats_init(&acc);
  for (int32_t k = 0; k < m->world; ++k) {  // rank order: exact and identical on every rank
    fognet_job_stats rec;
    memcpy(&rec, recs.data() + (size_t)k * sz, sz);
    fognet_job_stats_merge(&acc, &rec);
  }
  *inout = acc;
  return FOGNET_OK;
}

}  // extern "C"
