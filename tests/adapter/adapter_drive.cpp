// TEST INFRASTRUCTURE ONLY: drives integration/BrokerBaseAppHip (compiled
// against the stub in tests/adapter/stub) through the real libfognet_hip on a
// GPU.  A broker with N fog nodes receives a random stream of adverts (integer,
// fractional, NaN busy times; MIPS 0 for node 0 at first) and QoS-1 publishes;
// every task the adapter sends must go to the node the CPU oracle's
// restatement of BrokerBaseApp3.cc:267-281 (orc_decide_v3) picks on the view
// at that moment, and integer views must be decided once per view.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>

#include "BrokerBaseAppHip.cc"
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

struct Harness : BrokerBaseAppHip {
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
    int base() const { return baseSendPubAck; }
    const std::vector<Broker *> &view() const { return brokers; }
    ~Harness() {
        for (Broker *b : brokers) delete b;
    }
};

int main() {
    int failures = 0;
    long publishes = 0, views = 0;
    for (int scenario = 0; scenario < 6; ++scenario) {
        const int n = (int[]){1, 3, 5, 64, 257, 1000}[scenario];
        std::mt19937_64 rng(0x5EED + scenario);
        Harness h;
        h.setup(n);
        // node 0 advertises before the first publish (the reference divides by its MIPS)
        for (int j = 0; j < n; ++j) {
            FognetMsgAdvertiseMIPS *a = new FognetMsgAdvertiseMIPS("adv");
            a->setComputeBrokerID(h.ids[j].c_str());
            a->setMIPS(1000 * (1 + j % 4));
            a->setBusyTime(0.0);
            h.deliver(a);
            delete a;
        }
        long pubs = 0;
        int64_t views_here = 1;
        for (int step = 0; step < 3000; ++step) {
            g_now += 1000000000;
            if (rng() % 4 == 0) {  // an advert
                const int j = (int)(rng() % n);
                FognetMsgAdvertiseMIPS *a = new FognetMsgAdvertiseMIPS("adv");
                a->setComputeBrokerID(h.ids[j].c_str());
                a->setMIPS(1000 * (1 + j % 4));
                const int kind = (int)(rng() % 10);
                double b = (double)(rng() % 6);
                if (kind == 0) b += 0.5;            // fractional: decided per publish
                else if (kind == 1) b = NAN;        // never chosen
                else if (kind == 2) b += 1e-16;     // rounds away in busy + req/mips0
                a->setBusyTime(b);
                h.deliver(a);
                delete a;
                ++views_here;
                continue;
            }
            MqttMsgPublish *p = new MqttMsgPublish("pub");
            const int req = (int)(rng() % 64000);
            p->setMIPSRequired(req);
            p->setRequiredTime(0.01);
            p->setClientID("user");
            p->setMessageID(("m" + std::to_string(step)).c_str());
            const int sent0 = g_sent;
            h.deliver(p);
            delete p;
            ++pubs;
            std::vector<double> busy(n);
            std::vector<int32_t> mips(n);
            for (int j = 0; j < n; ++j) {
                busy[j] = h.view()[j]->getBusyTime();
                mips[j] = h.view()[j]->getMips();
            }
            int32_t want = -1;
            orc_decide_v3(n, busy.data(), mips.data(), req, &want);
            if (g_sent != sent0 + 1 || g_last_port != 2000 + want) {
                if (failures < 10)
                    fprintf(stderr, "scenario %d publish %ld: sent to port %d, oracle node %d\n", scenario, pubs,
                            g_last_port, want);
                ++failures;
            }
        }
        // at most one device call per publish, and integer views reuse one decision
        if (h.calls() > pubs || h.calls() < 1 || h.base() != 0) {
            fprintf(stderr, "scenario %d: %lld device calls for %ld publishes, %d base calls\n", scenario,
                    (long long)h.calls(), pubs, h.base());
            ++failures;
        }
        printf("scenario N=%d: %ld publishes, %lld device decisions, %lld views\n", n, pubs, (long long)h.calls(),
               (long long)views_here);
        publishes += pubs;
        views += views_here;
    }
    if (failures) {
        printf("adapter: %d failures\n", failures);
        return 1;
    }
    printf("adapter: all checks passed (%ld publishes over %ld views)\n", publishes, views);
    return 0;
}
