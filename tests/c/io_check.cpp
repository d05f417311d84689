// io_check.cpp — exercises the host I/O half of libfognet_hip (csrc/io.cpp:
// trace files, .sca/.vec writers, the mqttApp2 task source) for the
// AddressSanitizer / UBSan build (`make asan`), including truncated and
// corrupted trace files.  Exit 0 when every check passed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "fognet_io.h"

#define CHECK(c)                                                               \
  do {                                                                         \
    if (!(c)) {                                                                \
      std::fprintf(stderr, "io_check: %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, fognet_io_last_error()); \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string path = dir + "/io_check.fogntrc";
  const int R = 3, T = 257, N = 7;
  std::vector<int64_t> arrive(R * T), dl(R * N), ul(R * N), init(R * N);
  std::vector<int32_t> req(R * T), mips(R * N), ids(R * N);  // node_id [NR][N]
  std::vector<double> pb(R * N), pi(R * N);
  for (int i = 0; i < R * T; ++i) {
    arrive[i] = 1000000000000LL + 7919LL * i;
    req[i] = 1000 + i % 5000;
  }
  for (int j = 0; j < R * N; ++j) {
    mips[j] = 1000 * (1 + j % 4);
    dl[j] = ul[j] = init[j] = 1000000 + j;
    pb[j] = 10.0 + j;
    pi[j] = 3.5;
  }
  for (int j = 0; j < R * N; ++j) ids[j] = 100 + j % N;
  fognet_batch_in in{};
  in.R = R;
  in.T = T;
  in.N = N;
  in.node_stride = N;
  in.arrive_tick = arrive.data();
  in.req_mips = req.data();
  in.mips = mips.data();
  in.dl_tick = dl.data();
  in.ul_tick = ul.data();
  in.init_adv_tick = init.data();
  in.p_busy_w = pb.data();
  in.p_idle_w = pi.data();
  CHECK(fognet_trace_write(path.c_str(), &in, ids.data(), "io_check") == FOGNET_OK);

  fognet_trace_info info;
  CHECK(fognet_trace_info_read(path.c_str(), &info) == FOGNET_OK);
  CHECK(info.R == R && info.T == T && info.N == N && std::strcmp(info.note, "io_check") == 0);
  std::vector<int64_t> a2(R * T), d2(R * N), u2(R * N), i2(R * N);
  std::vector<int32_t> r2(R * T), m2(R * N), id2(R * N);
  std::vector<double> pb2(R * N), pi2(R * N);
  fognet_batch_in out{};
  out.arrive_tick = a2.data();
  out.req_mips = r2.data();
  out.mips = m2.data();
  out.dl_tick = d2.data();
  out.ul_tick = u2.data();
  out.init_adv_tick = i2.data();
  out.p_busy_w = pb2.data();
  out.p_idle_w = pi2.data();
  CHECK(fognet_trace_read(path.c_str(), &out, id2.data()) == FOGNET_OK);
  CHECK(a2 == arrive && r2 == req && m2 == mips && d2 == dl && id2 == ids && pb2 == pb);

  // truncations and a flipped byte are rejected
  std::FILE* f = std::fopen(path.c_str(), "rb");
  CHECK(f != nullptr);
  std::vector<unsigned char> bytes;
  for (int c; (c = std::fgetc(f)) != EOF;) bytes.push_back((unsigned char)c);
  std::fclose(f);
  const std::string bad = dir + "/io_check_bad.fogntrc";
  for (size_t cut : {size_t(0), size_t(8), size_t(255), size_t(256), bytes.size() / 2, bytes.size() - 1}) {
    f = std::fopen(bad.c_str(), "wb");
    std::fwrite(bytes.data(), 1, cut, f);
    std::fclose(f);
    CHECK(fognet_trace_read(bad.c_str(), &out, nullptr) != FOGNET_OK);
  }
  bytes[bytes.size() - 3] ^= 0x40;
  f = std::fopen(bad.c_str(), "wb");
  std::fwrite(bytes.data(), 1, bytes.size(), f);
  std::fclose(f);
  CHECK(fognet_trace_read(bad.c_str(), &out, nullptr) != FOGNET_OK);
  CHECK(fognet_trace_read((dir + "/does_not_exist").c_str(), &out, nullptr) != FOGNET_OK);

  // result files
  fognet_job_stats job;
  std::memset(&job, 0, sizeof job);
  job.n_reps = 2;
  job.n_tasks = job.n_qtime = 5;
  job.queue_min_raw = -1000;
  job.queue_max_raw = 3000000000000000LL;
  job.queue_sum[0] = (uint64_t)-1000;  // signed: -1000 + ... (two's complement)
  job.queue_sum[1] = job.queue_sum[2] = ~(uint64_t)0;
  job.queue_sq[0] = 12345;
  job.resp_min_ticks = 1;
  job.resp_max_ticks = 99;
  job.resp_sum[0] = 200;
  job.resp_sq[0] = 20000;
  std::vector<int64_t> hist(FOGNET_HIST_METRICS * FOGNET_HIST_BINS, 3);
  CHECK(fognet_write_sca((dir + "/io_check.sca").c_str(), "r", "Net", &job, hist.data()) == FOGNET_OK);
  std::vector<int32_t> node(T);
  std::vector<uint8_t> status(T);
  std::vector<int64_t> start(T);
  for (int i = 0; i < T; ++i) {
    node[i] = i % N;
    status[i] = i % 3 ? 4 : 5;
    start[i] = arrive[i] + dl[node[i]] + 5 * (i % 3);
  }
  CHECK(fognet_write_vec((dir + "/io_check.vec").c_str(), "r", "Net", T, N, arrive.data(), dl.data(), node.data(),
                         status.data(), start.data(), ids.data()) == FOGNET_OK);
  node[7] = N;  // out of range: rejected, nothing read past the node table
  CHECK(fognet_write_vec((dir + "/io_check.vec").c_str(), "r", "Net", T, N, arrive.data(), dl.data(), node.data(),
                         status.data(), start.data(), ids.data()) != FOGNET_OK);

  // the reference task source: three users, 50-ms interval, 2 s
  const int64_t st[3] = {0, 1000000000LL, 2000000000LL}, iv[3] = {50000000000LL, 50000000000LL, 70000000000LL};
  const int64_t up[3] = {1000000000LL, 1000000000LL, 1000000000LL}, dn[3] = {1000000000LL, 1000000000LL, -1};
  const int32_t cap = 1000;
  std::vector<int64_t> ga(cap);
  std::vector<int32_t> gr(cap), gu(cap);
  int32_t nt = 0, nt2 = 0;
  CHECK(fognet_gen_trace_mqtt(1, 3, st, iv, up, dn, 2000000000000LL, 200, 701, cap, ga.data(), gr.data(), gu.data(),
                              &nt) == FOGNET_OK);
  CHECK(fognet_gen_trace_mqtt(1, 3, st, iv, up, dn, 2000000000000LL, 200, 701, 5, ga.data(), gr.data(), gu.data(),
                              &nt2) != FOGNET_OK);  // cap too small: refused, nothing written past it
  nt2 = nt;
  CHECK(nt2 == nt && nt > 0);
  for (int i = 1; i < nt; ++i) CHECK(ga[i] >= ga[i - 1]);
  for (int i = 0; i < nt; ++i) CHECK(gr[i] >= 200 && gr[i] <= 900);
  std::printf("io_check: ok (%d publishes)\n", nt);
  return 0;
}
