// BrokerBaseApp2Hip.cc — see BrokerBaseApp2Hip.h and INTEGRATION.md §1.
// Link: -L<repo>/fognetsimpp_amd -lfognet_hip -L/opt/rocm/lib -lamdhip64
#include "BrokerBaseApp2Hip.h"

#include <sstream>
#include <string>

#include "inet/applications/mqttapp/fognetMessages/FognetMsgTask_m.h"

namespace inet {

Define_Module(BrokerBaseApp2Hip);

void BrokerBaseApp2Hip::initialize(int stage)
{
    BrokerBaseApp2::initialize(stage);
    if (stage == INITSTAGE_LOCAL) {
        int rc = fognet_create(&ctx, (int)par("hipDevice"));
        if (rc != FOGNET_OK)
            throw cRuntimeError("fognet_create: %s", fognet_status_string(rc));
    }
}

BrokerBaseApp2Hip::~BrokerBaseApp2Hip()
{
    fognet_destroy(ctx);
}

void BrokerBaseApp2Hip::handleMessageWhenUp(cMessage *msg)
{
    // a publish leaves the MIPS view as it is; anything else may change it
    if (dynamic_cast<MqttMsgPublish *>(msg) == nullptr)
        cacheValid = false;
    BrokerBaseApp2::handleMessageWhenUp(msg);
}

// BrokerBaseApp2.h:57
void BrokerBaseApp2Hip::sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status)
{
    if (status || brokers.empty()) {
        // the broker's own pool (:237-262) and the "no compute resource available" reply (:275-286)
        // go to the base class unchanged
        BrokerBaseApp2::sendPubAck(msg, ip, port, status);
        return;
    }
    int32_t k = 0;
    if (cacheValid) {
        k = cachedNode;
    }
    else {
        const int32_t n = (int32_t)brokers.size();
        viewMips.resize(n);
        for (int32_t j = 0; j < n; ++j)
            viewMips[j] = brokers[j]->getMips();
        // :241-248 on the device; the broker's own MIPS is passed as it is, and a forwarded publish
        // has MIPSRequired >= it (:181), so the action is FORWARD or DROPPED and k the chosen node
        int32_t action = 0;
        int rc = fognet_decide_v2(ctx, n, viewMips.data(), MIPS, msg->getMIPSRequired(), &k, &action);
        ++decideCalls;
        if (rc != FOGNET_OK)
            throw cRuntimeError("fognet_decide_v2: %s", fognet_last_error(ctx));
        if (action != FOGNET_V2_FORWARD && action != FOGNET_V2_DROPPED)
            throw cRuntimeError("fognet_decide_v2: unexpected action %d for a forwarded publish", (int)action);
        cacheValid = true;
        cachedNode = k;
    }
    forward(msg, ip, port, k);
}

void BrokerBaseApp2Hip::forward(MqttMsgPublish *msg, L3Address ip, int port, int32_t k)
{
    // the request is kept whether or not the task is sent (:254-259), with its deadline
    Request *req = new Request(msg->getClientID(), msg->getMessageID(), ip, port, msg->getMIPSRequired(),
                               simTime().dbl() + msg->getRequiredTime(), true);
    req->setRequestId(msg->getMessageID());
    requests.push_back(req);
    if (msg->getMIPSRequired() < brokers[k]->getMips()) {  // :262
        std::ostringstream str;
        str << "request " << msg->getMIPSRequired() << " for " << msg->getRequiredTime() << " sec from "
            << brokers[k]->getBrokerId();
        FognetMsgTask *tsk = new FognetMsgTask(str.str().c_str());
        tsk->setByteLength(msg->getByteLength());
        tsk->setRequiredMIPS(msg->getMIPSRequired());
        tsk->setRequiredTime(msg->getRequiredTime());
        tsk->setRequestID(msg->getMessageID());
        const std::string id = std::to_string(getId());
        tsk->setClientID(id.c_str());
        socket.sendTo(tsk, brokers[k]->getBrokerIp(), brokers[k]->getBrokerPort());
    }
}

}  // namespace inet
