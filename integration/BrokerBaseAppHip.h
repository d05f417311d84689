// BrokerBaseAppHip — the OMNeT++ broker module that hands FogNetSim++'s
// allocation decision (BrokerBaseApp3::sendPubAck, status == false,
// src/mqttapp/BrokerBaseApp3.cc:265-304) to libfognet_hip (include/fognet_hip.h).
// Compiled inside the FogNetSim++ tree, next to BrokerBaseApp3 (OMNeT++ 4.6 +
// INET 3.3); this repository checks it against a minimal stub of the
// identifiers it touches (tests/adapter/, `-fsyntax-only` and a GPU driver).
#ifndef BROKERBASEAPPHIP_H
#define BROKERBASEAPPHIP_H

#include <vector>

#include "inet/applications/mqttapp/BrokerBaseApp3.h"
#include "fognet_hip.h"

namespace inet {

class BrokerBaseAppHip : public BrokerBaseApp3
{
  protected:
    fognet_ctx *ctx = nullptr;
    std::vector<double> viewBusy;    // Broker::busyTime of brokers[j], CONNECT order
    std::vector<int32_t> viewMips;   // Broker::MIPS
    // The view only changes when a message other than a publish reaches the
    // broker (adverts, BrokerBaseApp3.cc:123-130; CONNECTs, :99-121).  While it
    // is integer-valued (busyTime is a sum of integer tskTime seconds,
    // ComputeBrokerApp3.cc:276-279) the argmin of busy_j + req/mips_0 does not
    // depend on req (the same integer is added to every candidate, no
    // rounding), so one decision per view serves every publish until the next
    // advert: exact, and one device call per advert instead of per publish.
    bool cacheValid = false;
    int32_t cachedNode = 0;
    int64_t decideCalls = 0;         // device decisions made (diagnostic)

    virtual void initialize(int stage) override;
    virtual void handleMessageWhenUp(cMessage *msg) override;
    virtual void sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status) override;
    // :283-302: record the request and send the task to node k
    virtual void offload(MqttMsgPublish *msg, L3Address ip, int port, int32_t k);

  public:
    virtual ~BrokerBaseAppHip();
};

}  // namespace inet

#endif
