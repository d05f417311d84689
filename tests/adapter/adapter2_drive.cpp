// TEST INFRASTRUCTURE ONLY: drives integration/BrokerBaseApp2Hip (compiled
// against the stub in tests/adapter/stub) through the real libfognet_hip on a
// GPU.  A v2 broker with N fog nodes receives a random stream of adverts
// (MIPS values with ties, zeros and values at node 0's), releases of its own
// pool and QoS-1 publishes; every forwarded publish must be recorded, and its
// task sent to the node the CPU oracle's restatement of BrokerBaseApp2.cc:
// 241-262 (orc_decide_v2) picks on the view at that moment -- or not sent when
// that node's MIPS is too small -- and a view must be decided once.
#include <cstdio>
#include <random>
#include <string>

#include "BrokerBaseApp2Hip.cc"
#include "../../oracle/fognet_oracle.h"

namespace inet {
static int64 g_now = 0;
static int g_last_port = -1;
static int g_sent = 0;
SimTime simTime() {
    SimTime t;
    t.raw_ = g_now;
    return t;
}
void UDPSocket::sendTo(cPacket *msg, L3Address, int destPort) {
    if (dynamic_cast<FognetMsgTask *>(msg)) {
        g_last_port = destPort;
        ++g_sent;
    }
    delete msg;
}
}  // namespace inet

using namespace inet;

struct Harness : BrokerBaseApp2Hip {
    std::vector<std::string> ids;
    void setup(int n) {
        initialize(INITSTAGE_LOCAL);
        ids.reserve(n);  // Broker keeps the id's pointer
        for (int j = 0; j < n; ++j) {
            ids.push_back("node" + std::to_string(j));
            brokers.push_back(new Broker(ids.back().c_str(), L3Address(100 + j), 2000 + j, 0));
        }
    }
    void deliver(cMessage *m) { handleMessageWhenUp(m); }
    int64_t calls() const { return decideCalls; }
    int local() const { return baseLocal; }
    int noNodes() const { return baseNoNodes; }
    int own() const { return MIPS; }
    void release(int m) { MIPS += m; }
    size_t nreq() const { return requests.size(); }
    const std::vector<Broker *> &view() const { return brokers; }
    ~Harness() {
        for (Broker *b : brokers) delete b;
    }
};

int main() {
    int failures = 0;
    long forwarded = 0, sent = 0, dropped = 0;
    const int mips_vals[] = {0, 500, 1000, 1000, 2000, 3000, 4000};
    for (int scenario = 0; scenario < 7; ++scenario) {
        const int n = (int[]){0, 1, 2, 5, 64, 257, 1000}[scenario];
        std::mt19937_64 rng(0x5EED2 + scenario);
        Harness h;
        h.setup(n);
        for (int j = 0; j < n; ++j) {  // first adverts (the reference starts every view at MIPS 0)
            FognetMsgAdvertiseMIPS *a = new FognetMsgAdvertiseMIPS("adv");
            a->setComputeBrokerID(h.ids[j].c_str());
            a->setMIPS(mips_vals[rng() % 7]);
            h.deliver(a);
            delete a;
        }
        long fw = 0, views = 1, local = 0;
        for (int step = 0; step < 3000; ++step) {
            g_now += 1000000000;
            const int kind = (int)(rng() % 8);
            if (kind == 0 && n > 0) {  // an advert
                FognetMsgAdvertiseMIPS *a = new FognetMsgAdvertiseMIPS("adv");
                const int j = (int)(rng() % n);
                a->setComputeBrokerID(h.ids[j].c_str());
                a->setMIPS(mips_vals[rng() % 7]);
                h.deliver(a);
                delete a;
                ++views;
                continue;
            }
            if (kind == 1) {  // the broker's own pool releases a reservation (its RELEASERESOURCE timer)
                h.release((int)(rng() % 700));
                continue;
            }
            MqttMsgPublish *p = new MqttMsgPublish("pub");
            const int req = (int)(rng() % 5000);
            p->setMIPSRequired(req);
            p->setRequiredTime(0.01);
            p->setClientID("user");
            p->setMessageID(("m" + std::to_string(step)).c_str());
            const int own = h.own();
            const int sent0 = g_sent, local0 = h.local(), none0 = h.noNodes();
            const size_t nreq0 = h.nreq();
            h.deliver(p);
            delete p;
            std::vector<int32_t> mips(n);
            for (int j = 0; j < n; ++j) mips[j] = h.view()[j]->getMips();
            int32_t want = -1, act = 0;
            orc_decide_v2(n, n ? mips.data() : nullptr, own, req, &want, &act);
            bool ok;
            if (act == ORC_V2_LOCAL) {
                ok = h.local() == local0 + 1 && g_sent == sent0 && h.nreq() == nreq0;
                ++local;
            } else if (act == ORC_V2_NO_NODES) {
                ok = h.noNodes() == none0 + 1 && g_sent == sent0;
            } else {
                ++fw;
                ok = h.nreq() == nreq0 + 1;  // recorded either way (:254-259)
                if (act == ORC_V2_FORWARD) {
                    ok = ok && g_sent == sent0 + 1 && g_last_port == 2000 + want;
                    ++sent;
                } else {
                    ok = ok && g_sent == sent0;
                    ++dropped;
                }
            }
            if (!ok) {
                if (failures < 10)
                    fprintf(stderr, "scenario %d step %d: action %d node %d, sent %d->%d port %d\n", scenario, step,
                            (int)act, (int)want, sent0, g_sent, g_last_port);
                ++failures;
            }
        }
        // at most one device call per forwarded publish and per view
        if (h.calls() > fw || h.calls() > views || (fw > 0 && h.calls() < 1)) {
            fprintf(stderr, "scenario %d: %lld device calls for %ld forwarded publishes over %ld views\n", scenario,
                    (long long)h.calls(), fw, views);
            ++failures;
        }
        printf("scenario N=%d: %ld forwarded, %ld local, %lld device decisions, %ld views\n", n, fw, local,
               (long long)h.calls(), views);
        forwarded += fw;
    }
    if (failures) {
        printf("adapter2: %d failures\n", failures);
        return 1;
    }
    printf("adapter2: all checks passed (%ld forwarded: %ld sent, %ld dropped)\n", forwarded, sent, dropped);
    return 0;
}
