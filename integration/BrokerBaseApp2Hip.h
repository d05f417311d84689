// BrokerBaseApp2Hip — the OMNeT++ broker module that hands the v2 broker's
// forwarding decision (BrokerBaseApp2::sendPubAck, status == false,
// src/mqttapp/BrokerBaseApp2.cc:235-287; the module config C1's ini selects,
// simulations/example/wirelessNet.ini:56) to libfognet_hip (fognet_decide_v2,
// include/fognet_hip.h).  Compiled inside the FogNetSim++ tree next to
// BrokerBaseApp2 (OMNeT++ 4.6 + INET 3.3); this repository checks it against a
// minimal stub of the identifiers it touches (tests/adapter/, `-fsyntax-only`
// and a GPU driver), like BrokerBaseAppHip for the v3 broker.
#ifndef BROKERBASEAPP2HIP_H
#define BROKERBASEAPP2HIP_H

#include <vector>

#include "inet/applications/mqttapp/BrokerBaseApp2.h"
#include "fognet_hip.h"

namespace inet {

class BrokerBaseApp2Hip : public BrokerBaseApp2
{
  protected:
    fognet_ctx *ctx = nullptr;
    std::vector<int32_t> viewMips;   // Broker::MIPS of brokers[j], CONNECT order
    // The v2 choice -- the LAST node whose advertised MIPS exceeds node 0's
    // (:241-248, the threshold is never updated) -- reads only the MIPS view,
    // which changes only when a message other than a publish reaches the broker
    // (adverts :128-136, CONNECTs :100-108).  So one device decision per view
    // serves every forwarded publish until the next such message; whether the
    // task is sent (MIPSRequired < the chosen node's MIPS, :262) is checked per
    // publish.  Exact, and one device call per view instead of per publish.
    bool cacheValid = false;
    int32_t cachedNode = 0;
    int64_t decideCalls = 0;         // device decisions made (diagnostic)

    virtual void initialize(int stage) override;
    virtual void handleMessageWhenUp(cMessage *msg) override;
    virtual void sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status) override;
    // :254-272: record the request; send the task to node k if it fits its MIPS
    virtual void forward(MqttMsgPublish *msg, L3Address ip, int port, int32_t k);

  public:
    virtual ~BrokerBaseApp2Hip();
};

}  // namespace inet

#endif
