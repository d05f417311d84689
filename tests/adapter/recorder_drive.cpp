// TEST INFRASTRUCTURE ONLY: drives integration/BrokerBaseAppRec (compiled
// against the stub in tests/adapter/stub) with the message stream a FogNetSim++
// v3 broker sees, then replays the trace it wrote.
//
// A ground-truth scenario (node MIPS, link latencies, first-advert ticks, a
// publish trace) is run through the CPU oracle, whose per-task nodes and ticks
// give every message the broker receives, each at its arrival tick with the
// creation tick its sender gave it: the nodes' first adverts (ComputeBrokerApp3
// .cc:205-222), the QoS-1 publishes (plus QoS-0 ones, which the broker does not
// allocate, BrokerBaseApp3.cc:138-158), each task's status-4/5 ack from its node
// (sent when the task arrives, :282-313) and the completion adverts (:224-256).
// The recorder writes the trace at finish(); the driver reads it back
// (fognet_trace_read), checks it equals the ground truth field by field, and
// replays it with fognet_run_batch (GPU, unless argv[2] == "--no-gpu") and with
// the oracle: both must reproduce the ground truth's decisions and ticks.
//
//   recorder_drive <trace path> [--no-gpu]
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "BrokerBaseAppRec.cc"
#include "fognet_io.h"
#include "../../oracle/fognet_oracle.h"

namespace inet {
static int64 g_now = 0;
SimTime simTime() {
    SimTime t;
    t.raw_ = g_now;
    return t;
}
void UDPSocket::sendTo(cPacket *msg, L3Address, int) { delete msg; }
}  // namespace inet

using namespace inet;

struct Harness : BrokerBaseAppRec {
    std::vector<std::string> ids;
    void setup(int n, const char *path) {
        parTraceFile.stubSet(path);
        initialize(INITSTAGE_LOCAL);
        ids.reserve(n);  // Broker keeps the id's pointer
        for (int j = 0; j < n; ++j) {  // CONNECT order (BrokerBaseApp3.cc:99-121)
            ids.push_back("computeBroker" + std::to_string(j));
            brokers.push_back(new Broker(ids.back().c_str(), L3Address(100 + j), 2000 + j, 0));
        }
    }
    void deliver(int64_t tick, cMessage *m) {
        g_now = tick;
        handleMessageWhenUp(m);
        delete m;
    }
    void end() { finish(); }
    ~Harness() {
        for (Broker *b : brokers) delete b;
    }
};

struct Ev {
    int64_t tick;
    int order;  // stable order among equal ticks (FES insertion order of the scenario)
    cMessage *msg;
};

static int failures = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            ++failures;                        \
            if (failures < 20) {               \
                printf("FAIL %s: ", #c);       \
                printf(__VA_ARGS__);           \
                printf("\n");                  \
            }                                  \
        }                                      \
    } while (0)

static int scenario(int s, const char *path, bool gpu) {
    const int N = s == 0 ? 24 : 200;
    const int T = s == 0 ? 3000 : 6000;
    std::mt19937_64 rng(0x5EED0100 + s);
    const int64_t MS = 1000000000;  // ticks per ms
    std::vector<int32_t> mips(N);
    std::vector<int64_t> dl(N), ul(N), init(N);
    int64_t last_init = 0;
    for (int j = 0; j < N; ++j) {
        mips[j] = 1000 * (1 + j % 4);
        dl[j] = 1000000 + (int64_t)(rng() % 999000001);  // 1 us .. 1 ms
        ul[j] = 1000000 + (int64_t)(rng() % 999000001);
        init[j] = ul[j] + (int64_t)(rng() % 50) * MS;
        last_init = std::max(last_init, init[j]);
    }
    std::vector<int64_t> arrive(T);
    std::vector<int32_t> req(T);
    int64_t t = last_init + MS;
    for (int i = 0; i < T; ++i) {
        t += (int64_t)(rng() % (s == 0 ? 900 : 150)) * MS;
        arrive[i] = t;
        req[i] = 1000 + (int32_t)(rng() % 63001);  // service up to 64 s: the argmin moves
    }
    // ground truth: the oracle's DES of the reference on these inputs
    std::vector<int32_t> node(T);
    std::vector<uint8_t> status(T);
    std::vector<int64_t> start(T), done(T);
    orc_rep_stats st;
    if (orc_run_batch(1, T, N, 0, arrive.data(), req.data(), mips.data(), dl.data(), ul.data(), init.data(),
                      node.data(), status.data(), start.data(), done.data(), &st, 1) != 0 || st.status != 0) {
        printf("FAIL oracle ground truth (status %d)\n", st.status);
        return 1;
    }
    // the broker's message stream
    std::vector<Ev> ev;
    int order = 0;
    std::vector<bool> acked(N, false);
    for (int j = 0; j < N; ++j) {
        FognetMsgAdvertiseMIPS *a = new FognetMsgAdvertiseMIPS("advertiseMIPS");
        a->setComputeBrokerID(("computeBroker" + std::to_string(j)).c_str());
        a->setMIPS(mips[j]);
        a->setBusyTime(0.0);
        a->stubSetCreationTime(init[j] - ul[j]);
        a->setControlInfo(new UDPDataIndication(L3Address(100 + j)));
        ev.push_back({init[j], order++, a});
    }
    for (int i = 0; i < T; ++i) {
        MqttMsgPublish *p = new MqttMsgPublish("publish");
        p->setMessageID(("m" + std::to_string(i)).c_str());
        p->setQoS(1);
        p->setMIPSRequired(req[i]);
        ev.push_back({arrive[i], order++, p});
        if (i % 97 == 0) {  // a QoS-0 publish at the same tick: not allocated, not recorded
            MqttMsgPublish *q = new MqttMsgPublish("publish0");
            q->setMessageID(("q" + std::to_string(i)).c_str());
            q->setQoS(0);
            q->setMIPSRequired(777);
            ev.push_back({arrive[i], order++, q});
        }
        const int k = node[i];
        const int64_t a_k = arrive[i] + dl[k];  // the task reaches node k; its 4/5 ack leaves then
        MqttMsgPuback *ack = new MqttMsgPuback("ack");
        ack->setMessageID(("m" + std::to_string(i)).c_str());
        ack->setStatus(status[i]);
        ack->stubSetCreationTime(a_k);
        ack->setControlInfo(new UDPDataIndication(L3Address(100 + k)));
        ev.push_back({a_k + ul[k], order++, ack});
        acked[k] = true;
        FognetMsgAdvertiseMIPS *c = new FognetMsgAdvertiseMIPS("advertiseMIPS");  // completion advert
        c->setComputeBrokerID(("computeBroker" + std::to_string(k)).c_str());
        c->setMIPS(mips[k]);
        c->setBusyTime(1.0);
        c->stubSetCreationTime(done[i]);
        c->setControlInfo(new UDPDataIndication(L3Address(100 + k)));
        ev.push_back({done[i] + ul[k], order++, c});
    }
    std::stable_sort(ev.begin(), ev.end(), [](const Ev &x, const Ev &y) {
        return x.tick != y.tick ? x.tick < y.tick : x.order < y.order;
    });
    {
        Harness h;
        h.setup(N, path);
        for (const Ev &e : ev) h.deliver(e.tick, e.msg);
        h.end();  // writes the trace
    }
    // read it back
    fognet_trace_info info;
    if (fognet_trace_info_read(path, &info) != FOGNET_OK) {
        printf("FAIL trace header: %s\n", fognet_io_last_error());
        return 1;
    }
    CHECK(info.R == 1 && info.T == T && info.N == N && info.node_stride == 0, "R %d T %d N %d", info.R, info.T, info.N);
    CHECK(strstr(info.note, "BrokerBaseAppRec") != nullptr, "note '%s'", info.note);
    std::vector<int64_t> r_arrive(T), r_dl(N), r_ul(N), r_init(N);
    std::vector<int32_t> r_req(T), r_mips(N);
    fognet_batch_in rin;
    memset(&rin, 0, sizeof rin);
    rin.arrive_tick = r_arrive.data();
    rin.req_mips = r_req.data();
    rin.mips = r_mips.data();
    rin.dl_tick = r_dl.data();
    rin.ul_tick = r_ul.data();
    rin.init_adv_tick = r_init.data();
    if (fognet_trace_read(path, &rin, nullptr) != FOGNET_OK) {
        printf("FAIL trace read: %s\n", fognet_io_last_error());
        return 1;
    }
    CHECK(r_arrive == arrive, "publish ticks differ");
    CHECK(r_req == req, "MIPSRequired differs");
    CHECK(r_mips == mips, "node MIPS differ");
    CHECK(r_ul == ul, "uplink latencies differ");
    CHECK(r_init == init, "first-advert ticks differ");
    int idle = 0;
    for (int j = 0; j < N; ++j) {
        CHECK(r_dl[j] == (acked[j] ? dl[j] : ul[j]), "node %d dl %lld vs %lld (acked %d)", j, (long long)r_dl[j],
              (long long)dl[j], (int)acked[j]);
        idle += !acked[j];
    }
    // the recorded trace replayed: the oracle, and the device engine, give the ground truth
    std::vector<int32_t> o_node(T);
    std::vector<uint8_t> o_status(T);
    std::vector<int64_t> o_start(T), o_done(T);
    orc_rep_stats ost;
    orc_run_batch(1, T, N, 0, r_arrive.data(), r_req.data(), r_mips.data(), r_dl.data(), r_ul.data(), r_init.data(),
                  o_node.data(), o_status.data(), o_start.data(), o_done.data(), &ost, 1);
    CHECK(o_node == node && o_status == status && o_start == start && o_done == done, "oracle replay differs");
    CHECK(memcmp(&ost, &st, sizeof st) == 0, "oracle replay statistics differ");
    if (gpu) {
        fognet_ctx *ctx = nullptr;
        if (fognet_create(&ctx, 0) != FOGNET_OK) {
            printf("FAIL fognet_create\n");
            return 1;
        }
        std::vector<int32_t> g_node(T);
        std::vector<uint8_t> g_status(T);
        std::vector<int64_t> g_start(T), g_done(T);
        fognet_rep_stats gst;
        fognet_batch_out out;
        memset(&out, 0, sizeof out);
        out.node = g_node.data();
        out.status = g_status.data();
        out.start_tick = g_start.data();
        out.done_tick = g_done.data();
        out.stats = &gst;
        rin.R = 1;
        rin.T = T;
        rin.N = N;
        rin.policy = FOGNET_POLICY_REF_V3;
        const int rc = fognet_run_batch(ctx, &rin, &out);
        CHECK(rc == FOGNET_OK, "fognet_run_batch: %s", fognet_last_error(ctx));
        CHECK(g_node == node && g_status == status && g_start == start && g_done == done, "device replay differs");
        CHECK(sizeof gst == sizeof st && memcmp(&gst, &st, sizeof st) == 0, "device statistics differ");
        fognet_destroy(ctx);
    }
    printf("scenario %d: N %d, T %d (+%d QoS-0), %d nodes never acked, %zu broker messages recorded\n", s, N, T,
           (T + 96) / 97, idle, ev.size());
    return 0;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        printf("usage: recorder_drive <trace path> [--no-gpu]\n");
        return 2;
    }
    const bool gpu = !(argc > 2 && strcmp(argv[2], "--no-gpu") == 0);
    for (int s = 0; s < 2; ++s)
        if (scenario(s, argv[1], gpu)) return 1;
    if (failures) {
        printf("recorder: %d failures\n", failures);
        return 1;
    }
    printf("recorder: all checks passed%s\n", gpu ? "" : " (no GPU replay)");
    return 0;
}
