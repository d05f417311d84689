// io.cpp — host-side formats of libfognet_hip (include/fognet_io.h): binary
// SoA trace files, OMNeT++ 4.6 .sca/.vec result files, and the reference's
// task source (mqttApp2's glibc-rand publish stream).  Plain host C++: no
// device code, no fognet_ctx.
#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <queue>
#include <string>
#include <vector>

#include "fognet_io.h"

namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
}

// ---------------------------------------------------------------- trace files

struct Header {
  char magic[8];
  uint32_t version, header_bytes;
  int32_t R, T, N, node_stride;
  uint32_t flags, reserved;
  uint64_t payload_bytes, checksum;
  char note[FOGNET_TRACE_NOTE_BYTES];
};
static_assert(sizeof(Header) <= FOGNET_TRACE_HEADER_BYTES, "header fits its block");

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
  const unsigned char* b = (const unsigned char*)p;
  for (size_t i = 0; i < n; ++i) {
    h ^= b[i];
    h *= 0x100000001b3ull;
  }
  return h;
}
constexpr uint64_t kFnvBasis = 0xcbf29ce484222325ull;

size_t align_up(size_t x) { return (x + FOGNET_TRACE_ALIGN - 1) & ~(size_t)(FOGNET_TRACE_ALIGN - 1); }

// The payload sections in file order (sizes from the header fields).
std::vector<size_t> section_sizes(int32_t R, int32_t T, int32_t N, int32_t stride, uint32_t flags) {
  const size_t NR = stride ? (size_t)R : 1u, nn = NR * (size_t)N, tt = (size_t)R * (size_t)T;
  std::vector<size_t> s = {nn * 4, nn * 8, nn * 8, nn * 8};
  s.push_back((flags & FOGNET_TRACE_FLAG_NODE_ID) ? nn * 4 : 0);
  s.push_back((flags & FOGNET_TRACE_FLAG_POWER) ? nn * 8 : 0);
  s.push_back((flags & FOGNET_TRACE_FLAG_POWER) ? nn * 8 : 0);
  s.push_back(tt * 8);
  s.push_back(tt * 4);
  return s;
}

size_t payload_bytes_of(const std::vector<size_t>& sizes) {
  size_t off = FOGNET_TRACE_HEADER_BYTES;
  for (size_t b : sizes) off = align_up(off) + b;
  return off - FOGNET_TRACE_HEADER_BYTES;
}

bool write_all(FILE* f, const void* p, size_t n) { return n == 0 || fwrite(p, 1, n, f) == n; }

int check_dims(int32_t R, int32_t T, int32_t N, int32_t stride) {
  if (R < 0 || T < 0 || N <= 0) return fail(FOGNET_ERR_ARG, "trace: need R >= 0, T >= 0, N > 0");
  if (stride != 0 && stride != N) return fail(FOGNET_ERR_ARG, "trace: node_stride must be 0 or N");
  return FOGNET_OK;
}

int read_header(FILE* f, const char* path, Header* h) {
  unsigned char blk[FOGNET_TRACE_HEADER_BYTES];
  if (fread(blk, 1, sizeof blk, f) != sizeof blk) return fail(FOGNET_ERR_ARG, std::string("trace: short header in ") + path);
  memcpy(h, blk, sizeof *h);
  if (memcmp(h->magic, FOGNET_TRACE_MAGIC, 8) != 0) return fail(FOGNET_ERR_ARG, std::string("trace: bad magic in ") + path);
  if (h->version != FOGNET_TRACE_VERSION) return fail(FOGNET_ERR_UNSUPPORTED, "trace: unsupported version");
  if (h->header_bytes != FOGNET_TRACE_HEADER_BYTES) return fail(FOGNET_ERR_ARG, "trace: bad header size");
  int rc = check_dims(h->R, h->T, h->N, h->node_stride);
  if (rc) return rc;
  if (h->flags & ~(FOGNET_TRACE_FLAG_POWER | FOGNET_TRACE_FLAG_NODE_ID)) return fail(FOGNET_ERR_UNSUPPORTED, "trace: unknown flags");
  const size_t want = payload_bytes_of(section_sizes(h->R, h->T, h->N, h->node_stride, h->flags));
  if (h->payload_bytes != want) return fail(FOGNET_ERR_ARG, "trace: payload size does not match the header");
  if (fseek(f, 0, SEEK_END) != 0) return fail(FOGNET_ERR_ARG, "trace: cannot seek");
  const long len = ftell(f);
  if (len < 0 || (uint64_t)len != FOGNET_TRACE_HEADER_BYTES + want)
    return fail(FOGNET_ERR_ARG, std::string("trace: file length does not match the header (truncated?): ") + path);
  if (fseek(f, FOGNET_TRACE_HEADER_BYTES, SEEK_SET) != 0) return fail(FOGNET_ERR_ARG, "trace: cannot seek");
  return FOGNET_OK;
}

// ---------------------------------------------------------------- exact moments

// Unsigned multi-limb integers (little-endian u64 limbs) for the exact
// variance numerator n*Q - S^2 (S, Q: 192-bit job sums, n < 2^63).
struct Big {
  uint64_t l[7] = {0, 0, 0, 0, 0, 0, 0};
};

Big big_of(const uint64_t* x, int n) {
  Big b;
  for (int i = 0; i < n; ++i) b.l[i] = x[i];
  return b;
}

Big big_mul(const Big& a, const Big& b) {
  Big r;
  for (int i = 0; i < 7; ++i) {
    unsigned __int128 carry = 0;
    for (int j = 0; i + j < 7; ++j) {
      const unsigned __int128 cur = (unsigned __int128)a.l[i] * b.l[j] + r.l[i + j] + carry;
      r.l[i + j] = (uint64_t)cur;
      carry = cur >> 64;
    }
  }
  return r;
}

bool big_ge(const Big& a, const Big& b) {
  for (int i = 6; i >= 0; --i)
    if (a.l[i] != b.l[i]) return a.l[i] > b.l[i];
  return true;
}

Big big_sub(const Big& a, const Big& b) {  // a >= b
  Big r;
  uint64_t borrow = 0;
  for (int i = 0; i < 7; ++i) {
    const unsigned __int128 d = (unsigned __int128)a.l[i] - b.l[i] - borrow;
    r.l[i] = (uint64_t)d;
    borrow = (uint64_t)(d >> 64) ? 1u : 0u;
  }
  return r;
}

long double big_ld(const Big& a) {
  long double v = 0.0L;
  for (int i = 6; i >= 0; --i) v = v * 18446744073709551616.0L + (long double)a.l[i];
  return v;
}

struct Moments {
  int64_t count;
  double mean, stddev, sum, sqrsum, min, max;  // ms
};

// count/mean/stddev/sum/sqrsum/min/max in ms of integer values given by their
// exact sum S (192-bit, two's complement if `sgn`) and sum of squares Q
// (cStdDev's fields, unbiased stddev).  ms_per_unit: 1e-9 for tick values,
// 1e-12 for raw emitted ms signals (the recorded value is raw * 1e-12, dbl()).
Moments moments(int64_t n, const uint64_t* S, const uint64_t* Q, int64_t mn, int64_t mx, bool sgn,
                bool raw_units) {
  Moments m;
  m.count = n;
  Big sa = big_of(S, 3);
  bool neg = false;
  if (sgn && (int64_t)S[2] < 0) {  // |S| by two's complement negation
    neg = true;
    const Big zero;
    Big ext = sa;
    for (int i = 3; i < 7; ++i) ext.l[i] = ~(uint64_t)0;
    sa = big_sub(zero, ext);
  }
  const long double unit = raw_units ? 1e-12L : 1e-9L;
  const long double s = (neg ? -1.0L : 1.0L) * big_ld(sa), q = big_ld(big_of(Q, 3));
  m.sum = (double)(s * unit);
  m.sqrsum = (double)(q * unit * unit);
  if (n == 0) {
    m.mean = m.stddev = m.min = m.max = NAN;
    return m;
  }
  m.mean = (double)(s / (long double)n * unit);
  m.min = raw_units ? (double)mn * 1e-12 : (double)mn / 1e9;  // raw: exactly the recorded dbl()
  m.max = raw_units ? (double)mx * 1e-12 : (double)mx / 1e9;
  if (n < 2) {
    m.stddev = NAN;  // cStdDev: variance undefined for a single value
    return m;
  }
  const uint64_t nn[1] = {(uint64_t)n};
  const Big nq = big_mul(big_of(nn, 1), big_of(Q, 3));
  const Big s2 = big_mul(sa, sa);
  const long double num = big_ge(nq, s2) ? big_ld(big_sub(nq, s2)) : 0.0L;
  const long double var = num / ((long double)n * (long double)(n - 1));
  m.stddev = (double)(sqrtl(var) * unit);
  return m;
}

// OMNeT++ 4.6 SimTime::toInt64 and the queueTime emission (replay_common.h
// qtime_raw, the host twin; x86-64 SSE2 doubles, no contraction).
bool simtime_to_int64(double x, int64_t* out) {
  const double f = floor(x + 0.5);
  if (!(fabs(f) < 9223372036854775808.0)) return false;
  *out = (int64_t)f;
  return true;
}

bool qtime_raw(int64_t now, int64_t a, int64_t* raw) {
  int64_t qs = 0;
  simtime_to_int64(1e12 * ((double)a * 1e-12), &qs);
  return simtime_to_int64((double)(now - qs) * 1000.0, raw);
}

// OMNeT++ number formatting (%.14g; NaN printed as "-nan" like cStdDev's 0/0).
std::string num(double v) {
  if (isnan(v)) return "-nan";
  if (isinf(v)) return v > 0 ? "inf" : "-inf";
  char b[64];
  snprintf(b, sizeof b, "%.14g", v);
  return b;
}

// simtime_t at scale 1e-12 as exact decimal seconds, trailing zeros trimmed.
std::string simtime_str(int64_t t) {
  const bool neg = t < 0;
  const uint64_t a = neg ? (uint64_t)0 - (uint64_t)t : (uint64_t)t;
  const uint64_t sec = a / (uint64_t)FOGNET_TICKS_PER_SECOND, frac = a % (uint64_t)FOGNET_TICKS_PER_SECOND;
  char b[64];
  if (frac == 0) {
    snprintf(b, sizeof b, "%s%llu", neg ? "-" : "", (unsigned long long)sec);
  } else {
    char f[16];
    snprintf(f, sizeof f, "%012llu", (unsigned long long)frac);
    int e = 11;
    while (e > 0 && f[e] == '0') f[e--] = '\0';
    snprintf(b, sizeof b, "%s%llu.%s", neg ? "-" : "", (unsigned long long)sec, f);
  }
  return b;
}

void run_header(FILE* f, const char* run_id, const char* network) {
  fprintf(f, "version 2\n");
  fprintf(f, "run %s\n", run_id);
  fprintf(f, "attr configname General\n");
  fprintf(f, "attr engine libfognet_hip\n");
  fprintf(f, "attr experiment General\n");
  fprintf(f, "attr iterationvars \"\"\n");
  fprintf(f, "attr iterationvars2 $repetition=0\n");
  fprintf(f, "attr measurement \"\"\n");
  fprintf(f, "attr network %s\n", network);
  fprintf(f, "attr repetition 0\n");
  fprintf(f, "attr replication #0\n");
  fprintf(f, "attr runnumber 0\n");
  fprintf(f, "attr seedset 0\n");
  fprintf(f, "\n");
}

void statistic(FILE* f, const std::string& module, const char* name, const char* kind, const Moments& m) {
  fprintf(f, "statistic %s \t%s:%s\n", module.c_str(), name, kind);
  fprintf(f, "field count %lld\n", (long long)m.count);
  fprintf(f, "field mean %s\n", num(m.mean).c_str());
  fprintf(f, "field stddev %s\n", num(m.stddev).c_str());
  fprintf(f, "field sum %s\n", num(m.sum).c_str());
  fprintf(f, "field sqrsum %s\n", num(m.sqrsum).c_str());
  fprintf(f, "field min %s\n", num(m.min).c_str());
  fprintf(f, "field max %s\n", num(m.max).c_str());
}

void stat_attrs(FILE* f, const char* name, const char* kind) {
  fprintf(f, "attr interpolationmode  none\n");
  fprintf(f, "attr source  %s\n", name);
  fprintf(f, "attr title  \"%s, %s\"\n", name, kind);
}

// ---------------------------------------------------------------- glibc rand()

// glibc random()/rand() with the default TYPE_3 state (degree 31, separation
// 3): r[0] = seed, r[i] = 16807 r[i-1] mod (2^31 - 1) for i < 31 (Schrage's
// method, as random_r.c), r[i] = r[i-31] for 31 <= i < 34, then
// r[i] = r[i-31] + r[i-3] mod 2^32; output k is r[k + 344] >> 1.
struct GlibcRand {
  uint32_t r[34];
  int i = 0;  // index (mod 34) of the next r[] to produce
  explicit GlibcRand(uint32_t seed) {
    int32_t w = seed == 0 ? 1 : (int32_t)seed;
    r[0] = (uint32_t)w;
    for (int k = 1; k < 31; ++k) {
      const int32_t hi = w / 127773, lo = w % 127773;
      w = 16807 * lo - 2836 * hi;
      if (w < 0) w += 2147483647;
      r[k] = (uint32_t)w;
    }
    for (int k = 31; k < 34; ++k) r[k] = r[k - 31];
    i = 34 % 34;
    for (int k = 34; k < 344; ++k) step();
  }
  uint32_t step() {  // produce r[n] for the next n (kept mod 34)
    const uint32_t v = r[(i + 34 - 31) % 34] + r[(i + 34 - 3) % 34];
    r[i] = v;
    i = (i + 1) % 34;
    return v;
  }
  int32_t next() { return (int32_t)(step() >> 1); }
};

}  // namespace

extern "C" {

const char* fognet_io_last_error(void) { return g_err.c_str(); }

int fognet_trace_write(const char* path, const fognet_batch_in* in, const int32_t* node_id, const char* note) {
  if (!path || !in) return fail(FOGNET_ERR_ARG, "trace_write: null argument");
  int rc = check_dims(in->R, in->T, in->N, in->node_stride);
  if (rc) return rc;
  if ((in->p_busy_w == nullptr) != (in->p_idle_w == nullptr))
    return fail(FOGNET_ERR_ARG, "trace_write: p_busy_w and p_idle_w must both be given or both be null");
  const bool tt = (size_t)in->R * (size_t)in->T > 0;
  if (!in->mips || !in->dl_tick || !in->ul_tick || !in->init_adv_tick || (tt && (!in->arrive_tick || !in->req_mips)))
    return fail(FOGNET_ERR_ARG, "trace_write: null array");
  Header h;
  memset(&h, 0, sizeof h);
  memcpy(h.magic, FOGNET_TRACE_MAGIC, 8);
  h.version = FOGNET_TRACE_VERSION;
  h.header_bytes = FOGNET_TRACE_HEADER_BYTES;
  h.R = in->R;
  h.T = in->T;
  h.N = in->N;
  h.node_stride = in->node_stride;
  h.flags = (in->p_busy_w ? FOGNET_TRACE_FLAG_POWER : 0u) | (node_id ? FOGNET_TRACE_FLAG_NODE_ID : 0u);
  if (note) strncpy(h.note, note, sizeof h.note - 1);
  const std::vector<size_t> sz = section_sizes(h.R, h.T, h.N, h.node_stride, h.flags);
  const void* src[9] = {in->mips, in->dl_tick, in->ul_tick, in->init_adv_tick, node_id,
                        in->p_busy_w, in->p_idle_w, in->arrive_tick, in->req_mips};
  h.payload_bytes = payload_bytes_of(sz);
  // checksum over the payload exactly as laid out in the file (padding = zeros)
  static const unsigned char zeros[FOGNET_TRACE_ALIGN] = {0};
  uint64_t ck = kFnvBasis;
  size_t off = FOGNET_TRACE_HEADER_BYTES;
  for (int s = 0; s < 9; ++s) {
    const size_t a = align_up(off);
    ck = fnv1a(ck, zeros, a - off);
    ck = fnv1a(ck, src[s], sz[s]);
    off = a + sz[s];
  }
  h.checksum = ck;
  FILE* f = fopen(path, "wb");
  if (!f) return fail(FOGNET_ERR_ARG, std::string("trace_write: cannot open ") + path);
  unsigned char blk[FOGNET_TRACE_HEADER_BYTES] = {0};
  memcpy(blk, &h, sizeof h);
  bool ok = write_all(f, blk, sizeof blk);
  off = FOGNET_TRACE_HEADER_BYTES;
  for (int s = 0; s < 9 && ok; ++s) {
    const size_t a = align_up(off);
    ok = write_all(f, zeros, a - off) && write_all(f, src[s], sz[s]);
    off = a + sz[s];
  }
  ok = (fclose(f) == 0) && ok;
  return ok ? FOGNET_OK : fail(FOGNET_ERR_ARG, std::string("trace_write: write failed: ") + path);
}

int fognet_trace_info_read(const char* path, fognet_trace_info* info) {
  if (!path || !info) return fail(FOGNET_ERR_ARG, "trace_info_read: null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(FOGNET_ERR_ARG, std::string("trace: cannot open ") + path);
  Header h;
  const int rc = read_header(f, path, &h);
  fclose(f);
  if (rc) return rc;
  info->R = h.R;
  info->T = h.T;
  info->N = h.N;
  info->node_stride = h.node_stride;
  info->flags = h.flags;
  info->version = h.version;
  info->payload_bytes = h.payload_bytes;
  info->checksum = h.checksum;
  memcpy(info->note, h.note, sizeof info->note);
  info->note[sizeof info->note - 1] = '\0';
  return FOGNET_OK;
}

int fognet_trace_read(const char* path, fognet_batch_in* out, int32_t* node_id) {
  if (!path || !out) return fail(FOGNET_ERR_ARG, "trace_read: null argument");
  FILE* f = fopen(path, "rb");
  if (!f) return fail(FOGNET_ERR_ARG, std::string("trace: cannot open ") + path);
  Header h;
  int rc = read_header(f, path, &h);
  if (rc) {
    fclose(f);
    return rc;
  }
  const bool pw = (h.flags & FOGNET_TRACE_FLAG_POWER) != 0, ids = (h.flags & FOGNET_TRACE_FLAG_NODE_ID) != 0;
  if ((out->p_busy_w && !pw) || (node_id && !ids)) {
    fclose(f);
    return fail(FOGNET_ERR_ARG, "trace_read: requested a section the file does not hold");
  }
  const bool tt = (size_t)h.R * (size_t)h.T > 0;
  if (!out->mips || !out->dl_tick || !out->ul_tick || !out->init_adv_tick || (tt && (!out->arrive_tick || !out->req_mips))) {
    fclose(f);
    return fail(FOGNET_ERR_ARG, "trace_read: null destination array");
  }
  const std::vector<size_t> sz = section_sizes(h.R, h.T, h.N, h.node_stride, h.flags);
  void* dst[9] = {(void*)out->mips, (void*)out->dl_tick, (void*)out->ul_tick, (void*)out->init_adv_tick, node_id,
                  (void*)out->p_busy_w, (void*)out->p_idle_w, (void*)out->arrive_tick, (void*)out->req_mips};
  uint64_t ck = kFnvBasis;
  size_t off = FOGNET_TRACE_HEADER_BYTES;
  std::vector<unsigned char> skip;
  bool ok = true;
  for (int s = 0; s < 9 && ok; ++s) {
    const size_t a = align_up(off);
    unsigned char pad[FOGNET_TRACE_ALIGN];
    ok = fread(pad, 1, a - off, f) == a - off;
    ck = fnv1a(ck, pad, a - off);
    if (ok && sz[s]) {
      void* d = dst[s];
      if (!d) {  // present in the file but not requested: read past it
        skip.resize(sz[s]);
        d = skip.data();
      }
      ok = fread(d, 1, sz[s], f) == sz[s];
      ck = fnv1a(ck, d, sz[s]);
    }
    off = a + sz[s];
  }
  fclose(f);
  if (!ok) return fail(FOGNET_ERR_ARG, std::string("trace_read: short read: ") + path);
  if (ck != h.checksum) return fail(FOGNET_ERR_ARG, std::string("trace_read: checksum mismatch (corrupt file): ") + path);
  out->R = h.R;
  out->T = h.T;
  out->N = h.N;
  out->node_stride = h.node_stride;
  return FOGNET_OK;
}

int fognet_write_sca(const char* path, const char* run_id, const char* network, const fognet_job_stats* job,
                     const int64_t* hist) {
  if (!path || !run_id || !network || !job) return fail(FOGNET_ERR_ARG, "write_sca: null argument");
  FILE* f = fopen(path, "w");
  if (!f) return fail(FOGNET_ERR_ARG, std::string("write_sca: cannot open ") + path);
  run_header(f, run_id, network);
  const std::string broker = std::string(network) + ".broker.udpApp[0]";
  const std::string nodes = std::string(network) + ".fogNodes.udpApp[0]";
  fprintf(f, "scalar %s \treplications \t%lld\n", broker.c_str(), (long long)job->n_reps);
  fprintf(f, "scalar %s \t\"failed replications\" \t%lld\n", broker.c_str(), (long long)job->n_failed);
  fprintf(f, "scalar %s \tdecisions \t%lld\n", broker.c_str(), (long long)job->n_tasks);
  fprintf(f, "scalar %s \t\"FES events\" \t%lld\n", broker.c_str(), (long long)job->events);
  fprintf(f, "scalar %s \t\"tasks queued\" \t%lld\n", nodes.c_str(), (long long)job->n_queued);
  fprintf(f, "scalar %s \t\"tasks started\" \t%lld\n", nodes.c_str(), (long long)job->n_started);
  fprintf(f, "scalar %s \t\"busy seconds\" \t%lld\n", nodes.c_str(), (long long)job->busy_s);
  fprintf(f, "scalar %s \t\"max pending\" \t%lld\n", nodes.c_str(), (long long)job->max_pending);
  fprintf(f, "scalar %s \t\"energy J\" \t%s\n", nodes.c_str(), num(job->energy_j).c_str());
  fprintf(f, "scalar %s \t\"makespan s\" \t%s\n", nodes.c_str(),
          job->n_tasks > 0 ? simtime_str(job->last_tick).c_str() : "-nan");
  fprintf(f, "scalar %s \t\"queueTime simtime overflows\" \t%lld\n", nodes.c_str(), (long long)job->n_qtime_overflow);
  fprintf(f, "scalar %s \t\"replications the reference aborts (queueTime overflow)\" \t%lld\n", nodes.c_str(),
          (long long)job->n_ref_aborted);
  const Moments q = moments(job->n_qtime, job->queue_sum, job->queue_sq, job->queue_min_raw, job->queue_max_raw, true, true);
  const Moments r = moments(job->n_tasks, job->resp_sum, job->resp_sq, job->resp_min_ticks, job->resp_max_ticks, false,
                            false);
  statistic(f, nodes, "queueTime", "stats", q);
  stat_attrs(f, "queueTime", "stats");
  statistic(f, broker, "response", "stats", r);
  stat_attrs(f, "response", "stats");
  if (hist) {
    const char* names[FOGNET_HIST_METRICS] = {"queueTime", "response"};
    const Moments* ms[FOGNET_HIST_METRICS] = {&q, &r};
    const std::string* mods[FOGNET_HIST_METRICS] = {&nodes, &broker};
    for (int m = 0; m < FOGNET_HIST_METRICS; ++m) {
      statistic(f, *mods[m], names[m], "histogram", *ms[m]);
      stat_attrs(f, names[m], "histogram");
      fprintf(f, "bin\t-INF\t0\n");
      for (int b = 0; b < FOGNET_HIST_BINS; ++b) {
        // bin 0: [0, 1) ms; bin b >= 1: [2^(b-1), 2^b) ms (fognet_hip.h)
        const double lo = b == 0 ? 0.0 : ldexp(1.0, b - 1);
        fprintf(f, "bin\t%s\t%lld\n", num(lo).c_str(), (long long)hist[m * FOGNET_HIST_BINS + b]);
      }
    }
  }
  const bool ok = ferror(f) == 0;
  return (fclose(f) == 0 && ok) ? FOGNET_OK : fail(FOGNET_ERR_ARG, std::string("write_sca: write failed: ") + path);
}

int fognet_write_vec(const char* path, const char* run_id, const char* network, int32_t T, int32_t N,
                     const int64_t* arrive_tick, const int64_t* dl_tick, const int32_t* node, const uint8_t* status,
                     const int64_t* start_tick, const int32_t* node_id) {
  if (!path || !run_id || !network || T < 0 || N <= 0) return fail(FOGNET_ERR_ARG, "write_vec: bad argument");
  if (T > 0 && (!arrive_tick || !dl_tick || !node || !status || !start_tick))
    return fail(FOGNET_ERR_ARG, "write_vec: null array");
  for (int32_t i = 0; i < T; ++i)
    if (node[i] < 0 || node[i] >= N) return fail(FOGNET_ERR_ARG, "write_vec: node index out of range");
  FILE* f = fopen(path, "w");
  if (!f) return fail(FOGNET_ERR_ARG, std::string("write_vec: cannot open ") + path);
  run_header(f, run_id, network);
  // vector ids: 0 = broker decisions, 1 + j = queueTime of node j
  fprintf(f, "vector 0  %s.broker.udpApp[0]  decision:vector  TV\n", network);
  fprintf(f, "attr interpolationmode  none\nattr source  decision\nattr title  \"decision, vector\"\n");
  for (int32_t j = 0; j < N; ++j) {
    fprintf(f, "vector %d  %s.fogNode[%d].udpApp[0]  queueTime:vector  TV\n", 1 + j, network,
            node_id ? node_id[j] : j);
    fprintf(f, "attr interpolationmode  none\nattr source  queueTime\nattr title  \"queueTime, vector\"\n");
  }
  for (int32_t i = 0; i < T; ++i) fprintf(f, "0\t%s\t%d\n", simtime_str(arrive_tick[i]).c_str(), node[i]);
  // per node in task order: FIFO, so each node's start ticks are nondecreasing
  std::vector<std::vector<int32_t>> per(N);
  for (int32_t i = 0; i < T; ++i)
    if (status[i] == 4) per[node[i]].push_back(i);
  for (int32_t j = 0; j < N; ++j)
    for (int32_t i : per[j]) {
      int64_t raw;  // the value ComputeBrokerApp3.cc:238 emits (fognet_hip.h "Reference signal values")
      if (!qtime_raw(start_tick[i], arrive_tick[i] + dl_tick[j], &raw)) continue;  // the reference throws
      fprintf(f, "%d\t%s\t%s\n", 1 + j, simtime_str(start_tick[i]).c_str(), num((double)raw * 1e-12).c_str());
    }
  const bool ok = ferror(f) == 0;
  return (fclose(f) == 0 && ok) ? FOGNET_OK : fail(FOGNET_ERR_ARG, std::string("write_vec: write failed: ") + path);
}

int fognet_gen_trace_mqtt(uint32_t seed, int32_t U, const int64_t* start_tick, const int64_t* interval_tick,
                          const int64_t* uplink_tick, const int64_t* downlink_tick, int64_t stop_tick,
                          int32_t req_base, int32_t req_span, int32_t cap, int64_t* arrive_tick, int32_t* req_mips,
                          int32_t* user_of, int32_t* out_T) {
  if (U < 0 || cap < 0 || req_span <= 0 || req_base < 0 || !out_T) return fail(FOGNET_ERR_ARG, "gen_trace_mqtt: bad argument");
  if (U > 0 && (!start_tick || !interval_tick || !uplink_tick || !downlink_tick))
    return fail(FOGNET_ERR_ARG, "gen_trace_mqtt: null user array");
  if (cap > 0 && (!arrive_tick || !req_mips)) return fail(FOGNET_ERR_ARG, "gen_trace_mqtt: null output array");
  for (int32_t u = 0; u < U; ++u)
    if (start_tick[u] < 0 || interval_tick[u] <= 0 || uplink_tick[u] < 0)
      return fail(FOGNET_ERR_ARG, "gen_trace_mqtt: need start >= 0, interval > 0, uplink >= 0");
  enum Kind { START, CONNECT_AT_BROKER, CONNACK, MQTTDATA };
  struct Ev {
    int64_t tick;
    uint64_t seq;
    int32_t kind, user;
    uint64_t gen;  // MQTTDATA: timer generation (cancelEvent invalidates older ones)
    bool operator>(const Ev& o) const { return tick != o.tick ? tick > o.tick : seq > o.seq; }
  };
  std::priority_queue<Ev, std::vector<Ev>, std::greater<Ev>> fes;
  uint64_t seq = 0;
  std::vector<uint64_t> gen(U, 0);
  for (int32_t u = 0; u < U; ++u) fes.push({start_tick[u], seq++, START, u, 0});  // handleNodeStart, user order
  GlibcRand rng(seed);
  struct Pub {
    int64_t at;
    int32_t req, user;
  };
  std::vector<Pub> pubs;
  auto arm = [&](int32_t u, int64_t now) {  // sendMqttData/processSend: re-arm only if < stop
    const int64_t d = now + interval_tick[u];
    if (d < stop_tick) {
      ++gen[u];  // cancelEvent(selfMsg)
      fes.push({d, seq++, MQTTDATA, u, gen[u]});
    }
  };
  auto publish = [&](int32_t u, int64_t now) {
    const int32_t req = req_base + rng.next() % req_span;  // mqttApp2.cc:370
    pubs.push_back({now + uplink_tick[u], req, u});
    arm(u, now);
  };
  while (!fes.empty()) {
    const Ev e = fes.top();
    fes.pop();
    switch (e.kind) {
      case START:
        fes.push({e.tick + uplink_tick[e.user], seq++, CONNECT_AT_BROKER, e.user, 0});
        arm(e.user, e.tick);
        break;
      case CONNECT_AT_BROKER:
        if (downlink_tick[e.user] >= 0) fes.push({e.tick + downlink_tick[e.user], seq++, CONNACK, e.user, 0});
        break;
      case CONNACK:
        publish(e.user, e.tick);
        break;
      case MQTTDATA:
        if (e.gen == gen[e.user]) publish(e.user, e.tick);
        break;
    }
  }
  // broker FES order: (arrival tick, send order); the send order is pubs' order
  std::vector<int32_t> idx(pubs.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = (int32_t)i;
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t a, int32_t b) { return pubs[a].at < pubs[b].at; });
  const size_t n = pubs.size();
  const size_t w = n < (size_t)cap ? n : (size_t)cap;
  for (size_t i = 0; i < w; ++i) {
    const Pub& p = pubs[idx[i]];
    arrive_tick[i] = p.at;
    req_mips[i] = p.req;
    if (user_of) user_of[i] = p.user;
  }
  *out_T = n > 0x7FFFFFFFu ? 0x7FFFFFFF : (int32_t)n;
  if (n > (size_t)cap) return fail(FOGNET_ERR_CAPACITY, "gen_trace_mqtt: more publishes than cap");
  return FOGNET_OK;
}

}  // extern "C"
