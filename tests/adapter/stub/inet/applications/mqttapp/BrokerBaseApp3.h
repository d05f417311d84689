// TEST INFRASTRUCTURE ONLY (see ../../../omnetpp_inet_stub.h): the members of
// BrokerBaseApp3 (src/mqttapp/BrokerBaseApp3.h:24-64) that the adapter uses,
// with the reference's types and access.  The handler bodies restate
// BrokerBaseApp3.cc:123-130 (advert: view update by CONNECT id) and :138-158
// (QoS-1 publish: sendPubAck(..., false)) for the GPU driver.
#pragma once
#include <cstring>

#include "../../../omnetpp_inet_stub.h"

namespace inet {

class BrokerBaseApp3 : public ApplicationBase {
  protected:
    UDPSocket socket;
    std::vector<Broker *> brokers;
    int MIPS = 0;
    std::vector<Request *> requests;
    int baseSendPubAck = 0;  // stub: calls that reached the base class's sendPubAck

    virtual void initialize(int stage) override {}
    virtual void handleMessageWhenUp(cMessage *msg) override {
        if (FognetMsgAdvertiseMIPS *a = dynamic_cast<FognetMsgAdvertiseMIPS *>(msg)) {
            for (unsigned j = 0; j < brokers.size(); j++)
                if (strcmp(brokers[j]->getBrokerId(), a->getComputeBrokerID()) == 0) {
                    brokers[j]->setMips(a->getMIPS());
                    brokers[j]->setBusyTime(a->getBusyTime());
                }
        } else if (MqttMsgPublish *p = dynamic_cast<MqttMsgPublish *>(msg)) {
            if (p->getQoS() == 1) sendPubAck(p, L3Address(1), 9, false);
        }
    }
    virtual void sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status) { ++baseSendPubAck; }
  public:
    virtual ~BrokerBaseApp3() {
        for (Request *r : requests) delete r;
    }
};

}  // namespace inet
