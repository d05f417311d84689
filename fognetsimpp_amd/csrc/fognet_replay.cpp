// fognet_replay — command-line trace-replay driver over libfognet_hip
// (caller 2: "the repo's own mini-DES trace-replay driver,
// which reads the same ini keys").  Host C++ only; the replay itself runs in
// the library's gfx950 kernels.
//
//   fognet_replay -f omnetpp.ini [-c Config] [--nodes N] [--users user[10],usr[10]] ...
//   fognet_replay --trace run.fogntrc --sca out.sca
//
// From the ini it reads the keys the reference modules read through par():
//   network                                      (module path prefix)
//   <net>.BaseBroker.udpApp[0].typename / MIPS   BrokerBaseApp3 -> FOGNET_POLICY_REF_V3 on
//                                                fognet_run_batch; BrokerBaseApp2 -> the v2
//                                                model replay (fognet_run_v2_dev)
//   <net>.ComputeBroker<k>.udpApp[0].MIPS        ComputeBrokerApp3.cc:43 / ComputeBrokerApp2
//   <net>.ComputeBroker<k>.udpApp[0].startTime   ComputeBrokerApp3.cc:54 (node CONNECT)
//   <net>.<user>.udpApp[0].sendInterval / startTime / stopTime   mqttApp2.cc:82-83, 203, 400
//   sim-time-limit                               (bounds the run)
// with OMNeT++ 4.x lookup rules: the selected [Config X] section first, then
// the sections it extends, then [General]; inside a section the first key
// (in file order) whose pattern matches the parameter's full path wins
// (`**` any string, `*` any string without '.', `?` one character except
// '.', `{a..b}` / `[a..b]` integer ranges).  Link latencies are INET's and are
// not in the ini: they are options (--dl/--ul node links, --user-ul/--user-dl).
// The publish trace is the reference task source (fognet_gen_trace_mqtt,
// mqttApp2.cc:198-409); replication r uses glibc srand(seed + r).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cctype>
#include <cinttypes>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "fognet_hip.h"
#include "fognet_io.h"

namespace {

constexpr int64_t kTick = 1;              // simtime_t raw unit: 1 ps
constexpr int64_t kMs = 1000000000LL;     // ticks per millisecond
constexpr int64_t kSec = 1000000000000LL;  // ticks per second
constexpr int64_t kNoTick = INT64_MIN;

[[noreturn]] void die(const std::string& msg) {
  std::fprintf(stderr, "fognet_replay: %s\n", msg.c_str());
  std::exit(2);
}

std::string trim(const std::string& s) {
  size_t a = 0, b = s.size();
  while (a < b && std::isspace((unsigned char)s[a])) ++a;
  while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
  return s.substr(a, b - a);
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  int depth = 0;  // commas inside [..] belong to the item
  for (char c : s) {
    if (c == '[') ++depth;
    if (c == ']') --depth;
    if (c == sep && depth == 0) {
      out.push_back(trim(cur));
      cur.clear();
    } else {
      cur += c;
    }
  }
  if (!trim(cur).empty()) out.push_back(trim(cur));
  return out;
}

// ---------------------------------------------------------------- omnetpp.ini

// OMNeT++ pattern match of a whole string (see the header comment).
bool parse_range(const std::string& p, size_t i, char close, size_t& end, long& lo, long& hi) {
  const size_t c = p.find(close, i);
  if (c == std::string::npos) return false;
  const std::string body = p.substr(i + 1, c - i - 1);
  const size_t dd = body.find("..");
  if (dd == std::string::npos) return false;
  const std::string a = trim(body.substr(0, dd)), b = trim(body.substr(dd + 2));
  char* e1 = nullptr;
  char* e2 = nullptr;
  lo = a.empty() ? 0 : std::strtol(a.c_str(), &e1, 10);
  hi = b.empty() ? LONG_MAX : std::strtol(b.c_str(), &e2, 10);
  if ((!a.empty() && *e1) || (!b.empty() && *e2)) return false;
  end = c + 1;
  return true;
}

bool match_at(const std::string& p, size_t pi, const std::string& s, size_t si) {
  while (pi < p.size()) {
    const char c = p[pi];
    if (c == '*') {
      const bool any = pi + 1 < p.size() && p[pi + 1] == '*';
      const size_t next = pi + (any ? 2 : 1);
      for (size_t k = si;; ++k) {
        if (match_at(p, next, s, k)) return true;
        if (k >= s.size() || (!any && s[k] == '.')) return false;
      }
    }
    if (c == '?') {
      if (si >= s.size() || s[si] == '.') return false;
      ++pi;
      ++si;
      continue;
    }
    if (c == '{' || (c == '[' && p.find("..", pi) < p.find(']', pi))) {
      size_t end = 0;
      long lo = 0, hi = 0;
      if (parse_range(p, pi, c == '{' ? '}' : ']', end, lo, hi)) {
        size_t k = si + (c == '[' ? 1 : 0);
        if (c == '[' && (si >= s.size() || s[si] != '[')) return false;
        const size_t d0 = k;
        while (k < s.size() && std::isdigit((unsigned char)s[k])) ++k;
        if (k == d0) return false;
        const long v = std::strtol(s.substr(d0, k - d0).c_str(), nullptr, 10);
        if (v < lo || v > hi) return false;
        if (c == '[') {
          if (k >= s.size() || s[k] != ']') return false;
          ++k;
        }
        pi = end;
        si = k;
        continue;
      }
    }
    if (si >= s.size() || s[si] != c) return false;
    ++pi;
    ++si;
  }
  return si == s.size();
}

bool pattern_match(const std::string& pattern, const std::string& s) { return match_at(pattern, 0, s, 0); }

struct IniEntry {
  std::string key, value, where;
};

struct IniSection {
  std::string name;  // "General" or the config name
  std::vector<std::string> extends;
  std::vector<IniEntry> entries;
};

class Ini {
 public:
  void load(const std::string& path, int depth = 0) {
    if (depth > 8) die("include nesting too deep at " + path);
    std::ifstream f(path);
    if (!f) die("cannot open " + path);
    const std::string dir = path.find('/') == std::string::npos ? "" : path.substr(0, path.rfind('/') + 1);
    std::string line, acc;
    int ln = 0, start = 0;
    while (std::getline(f, line)) {
      ++ln;
      if (acc.empty()) start = ln;
      // strip a comment outside quotes
      bool q = false;
      for (size_t i = 0; i < line.size(); ++i) {
        if (line[i] == '"') q = !q;
        if (line[i] == '#' && !q) {
          line.resize(i);
          break;
        }
      }
      std::string t = trim(line);
      if (!t.empty() && t.back() == '\\') {  // continuation
        acc += t.substr(0, t.size() - 1);
        continue;
      }
      acc += t;
      t = trim(acc);
      acc.clear();
      if (t.empty()) continue;
      const std::string where = path + ":" + std::to_string(start);
      if (t.front() == '[') {
        if (t.back() != ']') die("bad section header at " + where);
        std::string n = trim(t.substr(1, t.size() - 2));
        if (n.rfind("Config ", 0) == 0) n = trim(n.substr(7));
        secs_.push_back(IniSection{n, {}, {}});
        continue;
      }
      if (t.rfind("include ", 0) == 0) {
        load(dir + trim(t.substr(8)), depth + 1);
        continue;
      }
      const size_t eq = t.find('=');
      if (eq == std::string::npos) die("expected key = value at " + where);
      if (secs_.empty()) secs_.push_back(IniSection{"General", {}, {}});
      const std::string k = trim(t.substr(0, eq)), v = trim(t.substr(eq + 1));
      if (k == "extends") {
        for (const std::string& e : split(v, ',')) secs_.back().extends.push_back(e);
        continue;
      }
      secs_.back().entries.push_back(IniEntry{k, v, where});
    }
  }

  // Lookup order for a config: itself, the sections it extends (depth first),
  // then General.
  void select(const std::string& cfg) {
    chain_.clear();
    add_chain(cfg, 0);
    if (chain_.empty() && cfg != "General") die("no [Config " + cfg + "] section");
    if (cfg != "General") add_chain("General", 0);
  }

  // The first entry whose key pattern matches `full` (a module path + "." + parameter).
  const IniEntry* lookup(const std::string& full) const {
    for (const IniSection* s : chain_)
      for (const IniEntry& e : s->entries)
        if (pattern_match(e.key, full)) return &e;
    return nullptr;
  }

  // Option-style keys (network, sim-time-limit): exact key match.
  const IniEntry* option(const std::string& key) const {
    for (const IniSection* s : chain_)
      for (const IniEntry& e : s->entries)
        if (e.key == key) return &e;
    return nullptr;
  }

  // Highest k for which a key names `<prefix><k>` literally (no wildcard in that segment).
  int highest_literal_index(const std::string& prefix) const {
    int hi = 0;
    for (const IniSection* s : chain_)
      for (const IniEntry& e : s->entries) {
        size_t pos = 0;
        while ((pos = e.key.find(prefix, pos)) != std::string::npos) {
          size_t k = pos + prefix.size();
          const size_t d0 = k;
          while (k < e.key.size() && std::isdigit((unsigned char)e.key[k])) ++k;
          if (k > d0 && (k == e.key.size() || e.key[k] == '.'))
            hi = std::max(hi, std::atoi(e.key.substr(d0, k - d0).c_str()));
          pos = k;
        }
      }
    return hi;
  }

 private:
  void add_chain(const std::string& name, int depth) {
    if (depth > 16) die("extends chain too deep at " + name);
    for (const IniSection& s : secs_) {
      if (s.name != name) continue;
      if (std::find(chain_.begin(), chain_.end(), &s) == chain_.end()) chain_.push_back(&s);
    }
    for (const IniSection& s : secs_)
      if (s.name == name)
        for (const std::string& e : s.extends) add_chain(e, depth + 1);
  }

  std::vector<IniSection> secs_;
  std::vector<const IniSection*> chain_;
};

std::string unquote(const std::string& v) {
  if (v.size() >= 2 && v.front() == '"' && v.back() == '"') return v.substr(1, v.size() - 2);
  return v;
}

// A time value ("50ms", "1.5s", "0", "1000s") as exact ticks: the decimal
// digits are scaled in integers, so every value with <= 12 fractional
// digits of a second is exact (OMNeT++ would convert through a double).
int64_t parse_time(const std::string& raw, const std::string& what) {
  const std::string v = trim(unquote(raw));
  size_t i = 0;
  bool neg = false;
  if (i < v.size() && (v[i] == '-' || v[i] == '+')) neg = v[i++] == '-';
  __int128 mant = 0;
  int frac = -1;
  bool digits = false;
  for (; i < v.size(); ++i) {
    if (std::isdigit((unsigned char)v[i])) {
      mant = mant * 10 + (v[i] - '0');
      if (frac >= 0) ++frac;
      digits = true;
      if (mant > ((__int128)1 << 100)) die(what + ": value out of range: " + v);
    } else if (v[i] == '.' && frac < 0) {
      frac = 0;
    } else {
      break;
    }
  }
  if (!digits) die(what + ": not a constant time value (" + v + "); expressions and random variates are not supported");
  const std::string unit = trim(v.substr(i));
  __int128 scale;
  if (unit == "s" || unit.empty()) scale = kSec;
  else if (unit == "ms") scale = kMs;
  else if (unit == "us") scale = 1000000;
  else if (unit == "ns") scale = 1000;
  else if (unit == "ps") scale = kTick;
  else if (unit == "min") scale = 60 * kSec;
  else if (unit == "h") scale = 3600 * kSec;
  else if (unit == "d") scale = 86400 * kSec;
  else die(what + ": unknown time unit '" + unit + "' in " + v);
  __int128 t = mant * scale;
  for (int f = 0; f < std::max(frac, 0); ++f) {
    if (t % 10 != 0) die(what + ": " + v + " is not a whole number of ticks (1e-12 s)");
    t /= 10;
  }
  if (t > (__int128)((int64_t)1 << 61)) die(what + ": " + v + " exceeds 2^61 ticks");
  return neg ? -(int64_t)t : (int64_t)t;
}

int64_t parse_int(const std::string& raw, const std::string& what) {
  const std::string v = trim(unquote(raw));
  char* e = nullptr;
  const long long x = std::strtoll(v.c_str(), &e, 10);
  if (v.empty() || *e) die(what + ": not an integer constant: " + v);
  return x;
}

// ---------------------------------------------------------------- scenario

struct Options {
  std::string ini, config = "General", trace_in, trace_out, sca, vec, users = "user";
  std::string node_prefix = "ComputeBroker", comm_id;
  int world = 1, rank = 0;
  int nodes = 0, reps = 1, device = 0, ring = 0;
  uint32_t seed = 1;
  int64_t dl = kMs, ul = kMs, user_ul = kMs, user_dl = kMs, stop = kNoTick;
  bool user_dl_set = false, dry_run = false, policy_set = false, quiet = false, show = false;
  int policy = FOGNET_POLICY_REF_V3;
  double p_busy = -1.0, p_idle = -1.0;
};

struct Scenario {
  std::string network = "FogNet", broker_type = "BrokerBaseApp3";
  int32_t broker_mips = 0;
  std::vector<int32_t> mips;
  std::vector<int64_t> node_start;
  std::vector<std::string> users;
  std::vector<int64_t> u_start, u_interval;
  int64_t stop = kNoTick;
};

// "user" -> {user}; "user[3]" -> {user[0], user[1], user[2]}; comma-separated lists.
std::vector<std::string> expand_users(const std::string& spec) {
  std::vector<std::string> out;
  for (const std::string& item : split(spec, ',')) {
    const size_t b = item.find('[');
    if (b == std::string::npos) {
      out.push_back(item);
      continue;
    }
    const std::string base = item.substr(0, b);
    const int n = (int)parse_int(item.substr(b + 1, item.size() - b - 2), "--users " + item);
    for (int u = 0; u < n; ++u) out.push_back(base + "[" + std::to_string(u) + "]");
  }
  return out;
}

Scenario read_scenario(const Ini& ini, const Options& o) {
  Scenario sc;
  if (const IniEntry* e = ini.option("network")) sc.network = unquote(e->value);
  const std::string broker = sc.network + ".BaseBroker.udpApp[0].";
  if (const IniEntry* e = ini.lookup(broker + "typename")) sc.broker_type = unquote(e->value);
  if (const IniEntry* e = ini.lookup(broker + "MIPS")) sc.broker_mips = (int32_t)parse_int(e->value, e->where);
  const int n = o.nodes > 0 ? o.nodes : ini.highest_literal_index(o.node_prefix);
  if (n <= 0) die("cannot tell the number of fog nodes from the ini (no " + o.node_prefix + "<k> key): pass --nodes N");
  for (int k = 1; k <= n; ++k) {
    const std::string node = sc.network + "." + o.node_prefix + std::to_string(k) + ".udpApp[0].";
    const IniEntry* m = ini.lookup(node + "MIPS");
    if (!m) die("no MIPS for " + node + "MIPS");
    sc.mips.push_back((int32_t)parse_int(m->value, m->where));
    const IniEntry* st = ini.lookup(node + "startTime");
    sc.node_start.push_back(st ? parse_time(st->value, st->where) : 0);
  }
  int64_t stop = kNoTick;
  for (const std::string& u : expand_users(o.users)) {
    const std::string app = sc.network + "." + u + ".udpApp[0].";
    const IniEntry* iv = ini.lookup(app + "sendInterval");
    if (!iv) die("no sendInterval for " + app + "sendInterval (check --users)");
    const IniEntry* st = ini.lookup(app + "startTime");
    const IniEntry* sp = ini.lookup(app + "stopTime");
    sc.users.push_back(u);
    sc.u_interval.push_back(parse_time(iv->value, iv->where));
    sc.u_start.push_back(st ? parse_time(st->value, st->where) : 0);
    const int64_t s = sp ? parse_time(sp->value, sp->where) : kNoTick;
    if (s != kNoTick) {
      if (stop != kNoTick && s != stop)
        die("users have different stopTime values; the shared task source takes one: pass --stop");
      stop = s;
    }
  }
  if (const IniEntry* e = ini.option("sim-time-limit")) {
    const int64_t lim = parse_time(e->value, e->where);
    stop = stop == kNoTick ? lim : std::min(stop, lim);
  }
  if (o.stop != kNoTick) stop = o.stop;
  if (stop == kNoTick) die("no stopTime / sim-time-limit in the ini: pass --stop");
  sc.stop = stop;
  return sc;
}

void check(int rc, const char* what) {
  if (rc != FOGNET_OK) die(std::string(what) + ": " + fognet_status_string(rc) + " (" + fognet_io_last_error() + ")");
}

void check_ctx(fognet_ctx* ctx, int rc, const char* what) {
  if (rc != FOGNET_OK) die(std::string(what) + ": " + fognet_status_string(rc) + ": " + fognet_last_error(ctx));
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) die(std::string(what) + ": " + hipGetErrorString(e));
}

// The publish traces of R replications (glibc seeds seed .. seed + R - 1).
// Returns T (equal for every replication: the seed only changes MIPSRequired).
// Replications r0 .. r0 + n - 1 of the job (glibc seed o.seed + r).
int32_t gen_traces(const Scenario& sc, const Options& o, int64_t user_dl, int r0, int n, std::vector<int64_t>& arrive,
                   std::vector<int32_t>& req) {
  const int32_t U = (int32_t)sc.users.size();
  std::vector<int64_t> up(U, o.user_ul), dn(U, user_dl);
  // publishes per user <= (stop - start) / interval + 2 (the CONNACK publish)
  int64_t cap64 = 0;
  for (int u = 0; u < U; ++u) {
    if (sc.u_interval[u] <= 0) die("sendInterval must be > 0 for " + sc.users[u]);
    cap64 += std::max<int64_t>(0, (sc.stop - sc.u_start[u]) / sc.u_interval[u]) + 2;
  }
  if (cap64 > INT32_MAX) die("too many publishes for one replication");
  const int32_t cap = (int32_t)cap64;
  int32_t T = -1;
  std::vector<int64_t> a(cap);
  std::vector<int32_t> q(cap);
  for (int i = 0; i < n; ++i) {
    const int r = r0 + i;
    int32_t t = 0;
    check(fognet_gen_trace_mqtt(o.seed + (uint32_t)r, U, sc.u_start.data(), sc.u_interval.data(), up.data(), dn.data(),
                                sc.stop, 200, 701, cap, a.data(), q.data(), nullptr, &t),
          "fognet_gen_trace_mqtt");
    if (T < 0) {
      T = t;
      arrive.assign((size_t)n * T, 0);
      req.assign((size_t)n * T, 0);
    } else if (t != T) {
      die("replications produced different publish counts");
    }
    std::copy(a.begin(), a.begin() + T, arrive.begin() + (size_t)i * T);
    std::copy(q.begin(), q.begin() + T, req.begin() + (size_t)i * T);
  }
  return T;
}

void usage() {
  std::puts(
      "usage: fognet_replay (-f omnetpp.ini [-c Config] | --trace FILE) [options]\n"
      "  --nodes N            fog nodes ComputeBroker1..N (default: highest literal ComputeBroker<k> key)\n"
      "  --node-prefix P      node module name prefix (default ComputeBroker)\n"
      "  --users SPEC         user modules, e.g. user or user[10],usr[10] (default user)\n"
      "  --dl T --ul T        broker<->node one-way latencies (default 1ms)\n"
      "  --user-ul T          user->broker latency (default 1ms)\n"
      "  --user-dl T|none     broker->user latency of the CONNACK (default 1ms; none under BrokerBaseApp2)\n"
      "  --stop T             override stopTime / sim-time-limit\n"
      "  --reps R --seed S    replications, glibc srand seed of replication 0 (default 1 1)\n"
      "  --policy REF_V3|EXT_LAT   decision policy of a BrokerBaseApp3 run (default REF_V3)\n"
      "  --power BUSY,IDLE    node power model in W (builder-defined energy statistic)\n"
      "  --ring N             per-node pending capacity (power of two)\n"
      "  --trace-out FILE     write the FOGNTRC1 trace  --sca FILE / --vec FILE (replication 0)\n"
      "  --device D           HIP device (default 0)\n"
      "  --world W --rank K --comm-id FILE   one process per GPU: rank K replays its block of the\n"
      "                       --reps replications; the job statistics are exchanged over RCCL\n"
      "                       (fognet_allreduce_stats) and rank 0 writes the results; FILE carries\n"
      "                       the communicator id from rank 0 (a fresh path per run)\n"
      "  --dry-run            read the scenario and build the trace only (no GPU)\n"
      "  --show               print the resolved node and user parameters\n"
      "  --quiet              no summary on stdout");
}

Options parse_args(int argc, char** argv) {
  Options o;
  auto need = [&](int& i) -> std::string {
    if (i + 1 >= argc) die(std::string("missing value for ") + argv[i]);
    return argv[++i];
  };
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-f") o.ini = need(i);
    else if (a == "-c") o.config = need(i);
    else if (a == "--trace") o.trace_in = need(i);
    else if (a == "--trace-out") o.trace_out = need(i);
    else if (a == "--sca") o.sca = need(i);
    else if (a == "--vec") o.vec = need(i);
    else if (a == "--users") o.users = need(i);
    else if (a == "--node-prefix") o.node_prefix = need(i);
    else if (a == "--nodes") o.nodes = (int)parse_int(need(i), "--nodes");
    else if (a == "--reps") o.reps = (int)parse_int(need(i), "--reps");
    else if (a == "--seed") o.seed = (uint32_t)parse_int(need(i), "--seed");
    else if (a == "--device") o.device = (int)parse_int(need(i), "--device");
    else if (a == "--ring") o.ring = (int)parse_int(need(i), "--ring");
    else if (a == "--dl") o.dl = parse_time(need(i), "--dl");
    else if (a == "--ul") o.ul = parse_time(need(i), "--ul");
    else if (a == "--user-ul") o.user_ul = parse_time(need(i), "--user-ul");
    else if (a == "--user-dl") {
      const std::string v = need(i);
      o.user_dl = v == "none" ? -1 : parse_time(v, "--user-dl");
      o.user_dl_set = true;
    } else if (a == "--stop") o.stop = parse_time(need(i), "--stop");
    else if (a == "--policy") {
      const std::string v = need(i);
      if (v == "REF_V3") o.policy = FOGNET_POLICY_REF_V3;
      else if (v == "EXT_LAT") o.policy = FOGNET_POLICY_EXT_LAT;
      else die("--policy: REF_V3 or EXT_LAT");
      o.policy_set = true;
    } else if (a == "--power") {
      const std::vector<std::string> p = split(need(i), ',');
      if (p.size() != 2) die("--power BUSY,IDLE");
      o.p_busy = std::atof(p[0].c_str());
      o.p_idle = std::atof(p[1].c_str());
    } else if (a == "--dry-run") o.dry_run = true;
    else if (a == "--quiet") o.quiet = true;
    else if (a == "--show") o.show = true;
    else if (a == "--world") o.world = (int)parse_int(need(i), "--world");
    else if (a == "--rank") o.rank = (int)parse_int(need(i), "--rank");
    else if (a == "--comm-id") o.comm_id = need(i);
    else if (a == "-h" || a == "--help") {
      usage();
      std::exit(0);
    } else die("unknown option " + a + " (--help)");
  }
  if (o.ini.empty() == o.trace_in.empty()) die("give exactly one of -f INI and --trace FILE (--help)");
  if (o.reps <= 0) die("--reps must be > 0");
  if (o.world < 1 || o.rank < 0 || o.rank >= o.world) die("--world / --rank: need 0 <= rank < world");
  if (o.world > 1 && o.comm_id.empty()) die("--world > 1 needs --comm-id FILE (the communicator id's rendezvous)");
  if (o.reps < o.world) die("--reps must be >= --world (every rank replays a block of replications)");
  if (o.ring != 0 && (o.ring < 2 || o.ring > (1 << 15) || (o.ring & (o.ring - 1)) != 0))
    die("--ring must be a power of two in [2, 32768]");
  return o;
}

// ---------------------------------------------------------------- runs

// BrokerBaseApp3 + ComputeBrokerApp3 (the batch engine, host-buffer entry point).
// The job record of all ranks (fognet_allreduce_stats over the library's RCCL
// communicator); the 128-byte id goes from rank 0 to the others through the
// file o.comm_id (written atomically, removed once every rank has joined).
// Before any rank enters RCCL (whose communicator set-up waits for every rank
// without a timeout), the ranks agree through files o.comm_id + ".rank<k>"
// that every one of them finished its replay: a rank that failed (no device,
// a library error) writes "fail" instead of dying, and then no rank calls a
// collective.  Returns false if a rank failed or did not report within 300 s.
bool ranks_ready(const Options& o, bool local_ok) {
  auto name = [&](int k) { return o.comm_id + ".rank" + std::to_string(k); };
  const std::string tmp = name(o.rank) + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "w");
  if (!f || std::fputs(local_ok ? "ok" : "fail", f) < 0 || std::fclose(f) != 0 ||
      std::rename(tmp.c_str(), name(o.rank).c_str()) != 0)
    die("cannot write " + name(o.rank));
  bool all_ok = local_ok;
  for (int k = 0; k < o.world; ++k) {
    char buf[8] = {0};
    for (int waited = 0;; waited += 50) {
      FILE* g = std::fopen(name(k).c_str(), "r");
      if (g) {
        const size_t got = std::fread(buf, 1, sizeof buf - 1, g);
        std::fclose(g);
        if (got > 0) break;
      }
      if (waited > 300000) {
        std::fprintf(stderr, "fognet_replay: rank %d: no report from rank %d after 300 s\n", o.rank, k);
        return false;
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    if (std::strcmp(buf, "ok") != 0) {
      std::fprintf(stderr, "fognet_replay: rank %d: rank %d failed; skipping the statistics exchange\n", o.rank, k);
      all_ok = false;
    }
  }
  return all_ok;
}

void remove_rank_files(const Options& o) {
  for (int k = 0; k < o.world; ++k) std::remove((o.comm_id + ".rank" + std::to_string(k)).c_str());
}

void exchange_stats(const Options& o, fognet_ctx* ctx, fognet_job_stats* job, std::vector<int64_t>& hist) {
  uint8_t id[FOGNET_COMM_ID_BYTES];
  if (o.rank == 0) {
    check(fognet_comm_unique_id(id), "fognet_comm_unique_id");
    const std::string tmp = o.comm_id + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f || std::fwrite(id, 1, sizeof id, f) != sizeof id || std::fclose(f) != 0) die("cannot write " + tmp);
    if (std::rename(tmp.c_str(), o.comm_id.c_str()) != 0) die("cannot create " + o.comm_id);
  } else {
    for (int waited = 0;; waited += 50) {
      FILE* f = std::fopen(o.comm_id.c_str(), "rb");
      if (f) {
        const size_t got = std::fread(id, 1, sizeof id, f);
        std::fclose(f);
        if (got == sizeof id) break;
      }
      if (waited > 300000) die("no communicator id in " + o.comm_id + " after 300 s (is rank 0 running?)");
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
  }
  fognet_comm* comm = nullptr;
  check_ctx(ctx, fognet_comm_create(ctx, o.world, o.rank, id, &comm), "fognet_comm_create");
  if (o.rank == 0) {  // every rank has joined (and read every rank's report)
    std::remove(o.comm_id.c_str());
    remove_rank_files(o);
  }
  int64_t* d_hist = nullptr;
  const size_t hb = hist.size() * sizeof(int64_t);
  hip_check(hipMalloc((void**)&d_hist, hb), "hipMalloc");
  hip_check(hipMemcpy(d_hist, hist.data(), hb, hipMemcpyHostToDevice), "hipMemcpy");
  check_ctx(ctx, fognet_allreduce_stats(ctx, comm, job, d_hist, nullptr), "fognet_allreduce_stats");
  hip_check(hipMemcpy(hist.data(), d_hist, hb, hipMemcpyDeviceToHost), "hipMemcpy");
  (void)hipFree(d_hist);
  fognet_comm_destroy(comm);
}

int run_v3(const Options& o, fognet_batch_in in, const std::string& network, const std::string& run_id) {
  const size_t RT = (size_t)in.R * (size_t)in.T;
  std::vector<int32_t> node(RT);
  std::vector<uint8_t> status(RT);
  std::vector<int64_t> start(RT), done(RT), hist((size_t)FOGNET_HIST_METRICS * FOGNET_HIST_BINS, 0);
  std::vector<fognet_rep_stats> stats(in.R);
  fognet_batch_out out{node.data(), status.data(), start.data(), done.data(), stats.data(), nullptr, hist.data()};
  // status -1: "not replayed"; fognet_run_batch fails before any replay
  // (invalid batch, device error) or reports the first failed replication
  for (fognet_rep_stats& s : stats) s.status = -1;
  fognet_ctx* ctx = nullptr;
  std::string local_err;
  if (fognet_create(&ctx, o.device) != FOGNET_OK) {
    local_err = "fognet_create: no gfx950 device " + std::to_string(o.device);
    ctx = nullptr;
  } else {
    const int rc = fognet_run_batch(ctx, &in, &out);
    bool replayed = true;
    for (const fognet_rep_stats& s : stats) replayed = replayed && s.status != -1;
    if (rc != FOGNET_OK && !replayed)
      local_err = std::string("fognet_run_batch: ") + fognet_status_string(rc) + ": " + fognet_last_error(ctx);
  }
  if (o.comm_id.empty() && !local_err.empty()) die(local_err);
  if (!o.comm_id.empty()) {  // a failed rank reports instead of dying: no rank may be left in RCCL
    if (!local_err.empty()) std::fprintf(stderr, "fognet_replay: rank %d: %s\n", o.rank, local_err.c_str());
    if (!ranks_ready(o, local_err.empty())) {
      if (ctx) fognet_destroy(ctx);
      return 1;
    }
  }
  fognet_job_stats job;
  fognet_job_stats_init(&job);
  for (const fognet_rep_stats& s : stats) fognet_job_stats_add_rep(&job, &s);
  const int64_t local_failed = job.n_failed;
  if (!o.comm_id.empty()) exchange_stats(o, ctx, &job, hist);  // job + histogram of every rank
  if (o.rank != 0) {  // rank 0 writes the results
    fognet_destroy(ctx);
    return local_failed ? 1 : 0;
  }
  if (!o.sca.empty()) check(fognet_write_sca(o.sca.c_str(), run_id.c_str(), network.c_str(), &job, hist.data()), "sca");
  if (!o.vec.empty()) {  // replication 0's vectors (a failed replication has no complete outputs)
    if (stats[0].status != FOGNET_OK)
      die(std::string("--vec: replication 0 failed: ") + fognet_status_string(stats[0].status));
    check(fognet_write_vec(o.vec.c_str(), run_id.c_str(), network.c_str(), in.T, in.N, in.arrive_tick, in.dl_tick,
                           node.data(), status.data(), start.data(), nullptr),
          "vec");
  }
  if (!o.quiet) {
    std::printf("policy=%s R=%d T=%d N=%d decisions=%" PRId64 " queued=%" PRId64 " started=%" PRId64
                " failed_reps=%" PRId64 " makespan_ticks=%" PRId64 " max_pending=%" PRId64 "\n",
                in.policy == FOGNET_POLICY_EXT_LAT ? "EXT_LAT" : "REF_V3", in.R, in.T, in.N, job.n_tasks, job.n_queued,
                job.n_started, job.n_failed, job.last_tick, job.max_pending);
    std::vector<int64_t> per(in.N, 0);  // completed replications only (a failed one stops mid-trace)
    for (int32_t r = 0; r < in.R; ++r) {
      if (stats[r].status != FOGNET_OK) continue;
      for (size_t i = (size_t)r * in.T; i < (size_t)(r + 1) * in.T; ++i)
        if (node[i] >= 0 && node[i] < in.N) ++per[node[i]];
    }
    std::printf(o.world > 1 ? "tasks_per_node(rank 0)=" : "tasks_per_node=");
    for (int k = 0; k < in.N; ++k) std::printf("%s%" PRId64, k ? "," : "", per[k]);
    std::printf("\n");
    for (int r = 0; r < in.R; ++r)
      if (stats[r].status != FOGNET_OK)
        std::printf("replication %d: %s\n", r, fognet_status_string(stats[r].status));
  }
  fognet_destroy(ctx);
  return job.n_failed ? 1 : 0;
}

template <class T>
T* dev_copy(const std::vector<T>& h) {
  void* p = nullptr;
  hip_check(hipMalloc(&p, std::max<size_t>(1, h.size() * sizeof(T))), "hipMalloc");
  if (!h.empty()) hip_check(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
  return static_cast<T*>(p);
}

template <class T>
T* dev_alloc(size_t n) {
  void* p = nullptr;
  hip_check(hipMalloc(&p, std::max<size_t>(1, n * sizeof(T))), "hipMalloc");
  return static_cast<T*>(p);
}

// BrokerBaseApp2 + ComputeBrokerApp2 (the v2 model replay; device entry point).
int run_v2(const Options& o, const Scenario& sc, int32_t T, const std::vector<int64_t>& arrive,
           const std::vector<int32_t>& req, const std::vector<int64_t>& dl, const std::vector<int64_t>& ul,
           const std::vector<int64_t>& first_adv, const std::string& run_id) {
  const int32_t R = o.reps, N = (int32_t)sc.mips.size();
  if (N > FOGNET_V2_MAX_NODES) die("BrokerBaseApp2 replays take at most 16384 fog nodes");
  hip_check(hipSetDevice(o.device), "hipSetDevice");
  fognet_ctx* ctx = nullptr;
  if (fognet_create(&ctx, o.device) != FOGNET_OK) die("fognet_create: no gfx950 device " + std::to_string(o.device));
  std::vector<int32_t> bm(R, sc.broker_mips);
  std::vector<double> rt(R, 0.01);  // MqttMsgPublish.requiredTime (mqttApp2.cc:372)
  std::vector<int64_t> stop(R, sc.stop);
  fognet_v2_in in{};
  in.R = R;
  in.T = T;
  in.N = N;
  in.arrive_tick = dev_copy(arrive);
  in.req_mips = dev_copy(req);
  in.broker_mips = dev_copy(bm);
  in.required_time_s = dev_copy(rt);
  in.stop_tick = dev_copy(stop);
  in.mips = dev_copy(sc.mips);
  in.dl_tick = dev_copy(dl);
  in.ul_tick = dev_copy(ul);
  in.first_adv_tick = dev_copy(first_adv);
  const size_t RT = (size_t)R * T;
  fognet_v2_out out{dev_alloc<int32_t>(RT), dev_alloc<uint8_t>(RT), dev_alloc<int64_t>(RT), dev_alloc<int64_t>(RT),
                    dev_alloc<fognet_v2_stats>(R)};
  check_ctx(ctx, fognet_run_v2_dev(ctx, &in, &out, nullptr), "fognet_run_v2_dev");
  hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
  std::vector<fognet_v2_stats> st(R);
  std::vector<int32_t> node(RT);
  hip_check(hipMemcpy(st.data(), out.stats, R * sizeof(fognet_v2_stats), hipMemcpyDeviceToHost), "hipMemcpy");
  hip_check(hipMemcpy(node.data(), out.node, RT * sizeof(int32_t), hipMemcpyDeviceToHost), "hipMemcpy");
  fognet_v2_stats tot{};
  int failed = 0;
  for (const fognet_v2_stats& s : st) {
    tot.n_tasks += s.n_tasks;
    tot.n_local += s.n_local;
    tot.n_forwarded += s.n_forwarded;
    tot.n_accepted += s.n_accepted;
    tot.n_rejected += s.n_rejected;
    tot.n_dropped += s.n_dropped;
    tot.n_no_nodes += s.n_no_nodes;
    tot.events += s.events;
    failed += s.status != FOGNET_OK;
  }
  if (!o.sca.empty()) {  // BrokerBaseApp2 has no statistics of its own: the driver's scalars
    FILE* f = std::fopen(o.sca.c_str(), "w");
    if (!f) die("cannot write " + o.sca);
    std::fprintf(f, "version 2\nrun %s\nattr network %s\n\n", run_id.c_str(), sc.network.c_str());
    const std::string m = sc.network + ".BaseBroker.udpApp[0]";
    const std::pair<const char*, int64_t> rows[] = {
        {"publishes", tot.n_tasks},   {"servedLocally", tot.n_local}, {"forwarded", tot.n_forwarded},
        {"acceptedByNode", tot.n_accepted}, {"rejectedByNode", tot.n_rejected}, {"dropped", tot.n_dropped},
        {"noNodes", tot.n_no_nodes},  {"events", tot.events},         {"replications", R},
        {"failedReplications", failed}};
    for (const auto& r : rows) std::fprintf(f, "scalar %s \t%s \t%" PRId64 "\n", m.c_str(), r.first, r.second);
    std::fclose(f);
  }
  if (!o.quiet) {
    std::printf("model=v2 R=%d T=%d N=%d publishes=%" PRId64 " local=%" PRId64 " forwarded=%" PRId64
                " accepted=%" PRId64 " rejected=%" PRId64 " dropped=%" PRId64 " events=%" PRId64 " failed_reps=%d\n",
                R, T, N, tot.n_tasks, tot.n_local, tot.n_forwarded, tot.n_accepted, tot.n_rejected, tot.n_dropped,
                tot.events, failed);
    std::vector<int64_t> per(N, 0);
    for (size_t i = 0; i < (size_t)T; ++i)
      if (node[i] >= 0) ++per[node[i]];
    std::printf("forwarded_per_node(rep0)=");
    for (int k = 0; k < N; ++k) std::printf("%s%" PRId64, k ? "," : "", per[k]);
    std::printf("\n");
  }
  for (const void* p : {(const void*)in.arrive_tick, (const void*)in.req_mips, (const void*)in.broker_mips,
                        (const void*)in.required_time_s, (const void*)in.stop_tick, (const void*)in.mips,
                        (const void*)in.dl_tick, (const void*)in.ul_tick, (const void*)in.first_adv_tick,
                        (const void*)out.node, (const void*)out.status, (const void*)out.start_tick,
                        (const void*)out.done_tick, (const void*)out.stats})
    (void)hipFree(const_cast<void*>(p));
  fognet_destroy(ctx);
  return failed ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  const Options o = parse_args(argc, argv);
  const std::string run_id = o.trace_in.empty() ? o.config + "-0" : "trace-0";

  if (!o.trace_in.empty()) {  // replay a trace file (REF_V3 / EXT_LAT engine)
    if (o.world > 1) die("--trace replays run on one GPU (--world 1)");
    fognet_trace_info ti;
    check(fognet_trace_info_read(o.trace_in.c_str(), &ti), "trace header");
    const size_t NR = ti.node_stride ? (size_t)ti.R : 1, RT = (size_t)ti.R * (size_t)ti.T;
    std::vector<int64_t> arrive(RT), dl(NR * ti.N), ul(NR * ti.N), init(NR * ti.N);
    std::vector<int32_t> req(RT), mips(NR * ti.N);
    std::vector<double> pb, pi;
    fognet_batch_in in{};
    in.arrive_tick = arrive.data();
    in.req_mips = req.data();
    in.mips = mips.data();
    in.dl_tick = dl.data();
    in.ul_tick = ul.data();
    in.init_adv_tick = init.data();
    if (ti.flags & FOGNET_TRACE_FLAG_POWER) {
      pb.resize(NR * ti.N);
      pi.resize(NR * ti.N);
      in.p_busy_w = pb.data();
      in.p_idle_w = pi.data();
    }
    check(fognet_trace_read(o.trace_in.c_str(), &in, nullptr), "trace read");
    in.policy = o.policy;
    in.ring_capacity = o.ring;
    if (!o.quiet) std::printf("trace %s: R=%d T=%d N=%d note=\"%s\"\n", o.trace_in.c_str(), ti.R, ti.T, ti.N, ti.note);
    if (o.dry_run) return 0;
    return run_v3(o, in, "FogNet", run_id);
  }

  Ini ini;
  ini.load(o.ini);
  ini.select(o.config);
  const Scenario sc = read_scenario(ini, o);
  const bool v2 = sc.broker_type == "BrokerBaseApp2";
  if (!v2 && sc.broker_type != "BrokerBaseApp3" && sc.broker_type != "BrokerBaseAppHip")
    die("broker module " + sc.broker_type + " is not on the engine's path (BrokerBaseApp3, BrokerBaseApp2)");
  if (v2 && o.policy_set) die("--policy applies to BrokerBaseApp3 runs");
  const int32_t N = (int32_t)sc.mips.size();
  // BrokerBaseApp2 does not answer a user's CONNECT with a CONNACK, so its
  // users publish from startTime + sendInterval on
  const int64_t user_dl = o.user_dl_set ? o.user_dl : (v2 ? -1 : o.user_dl);
  std::vector<int64_t> arrive;
  std::vector<int32_t> req;
  // rank's contiguous block of the job's replications (the first reps % world ranks take one more)
  const int q = o.reps / o.world, rem = o.reps % o.world;
  const int r0 = o.rank * q + std::min(o.rank, rem), nr = q + (o.rank < rem ? 1 : 0);
  const int32_t T = gen_traces(sc, o, user_dl, r0, nr, arrive, req);

  // node k: CONNECT at startTime reaches the broker after ul, the CONNACK
  // comes back after dl, the first ADVERTISEMIPS fires 0.01 s later
  // (ComputeBrokerApp3.cc:261-267) and reaches the broker after ul
  std::vector<int64_t> dl(N, o.dl), ul(N, o.ul), first_adv(N), init(N);
  int64_t last_init = INT64_MIN;
  for (int k = 0; k < N; ++k) {
    first_adv[k] = sc.node_start[k] + o.ul + o.dl + 10 * kMs;
    init[k] = first_adv[k] + o.ul;
    last_init = std::max(last_init, init[k]);
  }
  if (!o.quiet)
    std::printf("scenario %s [%s]: network=%s broker=%s nodes=%d users=%zu stop=%.12g s publishes/rep=%d\n",
                o.ini.c_str(), o.config.c_str(), sc.network.c_str(), sc.broker_type.c_str(), N, sc.users.size(),
                (double)sc.stop / kSec, T);
  if (o.show) {
    std::printf("broker %s.BaseBroker.udpApp[0] %s MIPS=%d\n", sc.network.c_str(), sc.broker_type.c_str(), sc.broker_mips);
    for (int k = 0; k < N; ++k)
      std::printf("node %d %s%d MIPS=%d startTime_ticks=%" PRId64 " first_advert_at_broker_ticks=%" PRId64 "\n", k,
                  o.node_prefix.c_str(), k + 1, sc.mips[k], sc.node_start[k], init[k]);
    for (size_t u = 0; u < sc.users.size(); ++u)
      std::printf("user %s startTime_ticks=%" PRId64 " sendInterval_ticks=%" PRId64 "\n", sc.users[u].c_str(),
                  sc.u_start[u], sc.u_interval[u]);
    std::printf("stop_ticks=%" PRId64 "\n", sc.stop);
  }
  if (!v2 && T > 0 && arrive[0] <= last_init) {
    char buf[256];
    std::snprintf(buf, sizeof buf,
                  "the first publish reaches the broker at tick %" PRId64 ", before the last first advert (tick %" PRId64
                  "): BrokerBaseApp3 would divide by the unadvertised MIPS 0 (BrokerBaseApp3.cc:267); "
                  "delay the users (startTime, --user-dl) or speed up the nodes' links",
                  arrive[0], last_init);
    die(buf);
  }

  std::vector<double> pb, pi;
  fognet_batch_in in{};
  in.R = nr;
  in.T = T;
  in.N = N;
  in.policy = o.policy;
  in.node_stride = 0;
  in.ring_capacity = o.ring;
  in.arrive_tick = arrive.data();
  in.req_mips = req.data();
  in.mips = sc.mips.data();
  in.dl_tick = dl.data();
  in.ul_tick = ul.data();
  in.init_adv_tick = init.data();
  if (o.p_busy >= 0.0) {
    pb.assign(N, o.p_busy);
    pi.assign(N, o.p_idle);
    in.p_busy_w = pb.data();
    in.p_idle_w = pi.data();
  }
  if (!o.trace_out.empty()) {
    if (v2) die("--trace-out: trace files hold BrokerBaseApp3 inputs (first-advert arrival ticks)");
    check(fognet_trace_write(o.trace_out.c_str(), &in, nullptr, ("fognet_replay " + o.ini + " [" + o.config + "]").c_str()),
          "trace write");
  }
  if (o.dry_run) return 0;
  if (v2) {
    if (o.world > 1) die("BrokerBaseApp2 replays run on one GPU (--world 1)");
    return run_v2(o, sc, T, arrive, req, dl, ul, first_adv, run_id);
  }
  return run_v3(o, in, sc.network, run_id);
}
