// TEST INFRASTRUCTURE ONLY (see ../../../omnetpp_inet_stub.h): the members of
// BrokerBaseApp2 (src/mqttapp/BrokerBaseApp2.h:27-60) that the v2 adapter uses,
// with the reference's types and access.  The handler bodies restate
// BrokerBaseApp2.cc:128-136 (advert: MIPS view update by CONNECT id) and
// :178-198 (QoS-1 publish: local when MIPSRequired < MIPS, else forwarded) for
// the GPU driver; the base sendPubAck only counts and reserves (:235-240).
#pragma once
#include <cstring>

#include "../../../omnetpp_inet_stub.h"

namespace inet {

class BrokerBaseApp2 : public ApplicationBase {
  protected:
    UDPSocket socket;
    std::vector<Broker *> brokers;
    int MIPS = 1000;
    std::vector<Request *> requests;
    int baseLocal = 0, baseNoNodes = 0;  // stub: calls that reached the base class's sendPubAck

    virtual void initialize(int stage) override {}
    virtual void handleMessageWhenUp(cMessage *msg) override {
        if (FognetMsgAdvertiseMIPS *a = dynamic_cast<FognetMsgAdvertiseMIPS *>(msg)) {
            for (unsigned j = 0; j < brokers.size(); j++)
                if (strcmp(brokers[j]->getBrokerId(), a->getComputeBrokerID()) == 0) brokers[j]->setMips(a->getMIPS());
        } else if (MqttMsgPublish *p = dynamic_cast<MqttMsgPublish *>(msg)) {
            if (p->getQoS() == 1) sendPubAck(p, L3Address(1), 9, p->getMIPSRequired() < MIPS);
        }
    }
    virtual void sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status) {
        if (status) {
            ++baseLocal;
            MIPS = MIPS - msg->getMIPSRequired();
        } else {
            ++baseNoNodes;
        }
    }
  public:
    virtual ~BrokerBaseApp2() {
        for (Request *r : requests) delete r;
    }
};

}  // namespace inet
