// BrokerBaseAppHip.cc — see BrokerBaseAppHip.h and INTEGRATION.md §1.
// Link: -L<repo>/fognetsimpp_amd -lfognet_hip -L/opt/rocm/lib -lamdhip64
#include "BrokerBaseAppHip.h"

#include <cmath>
#include <sstream>
#include <string>

#include "inet/applications/mqttapp/fognetMessages/FognetMsgTask_m.h"

namespace inet {

Define_Module(BrokerBaseAppHip);

void BrokerBaseAppHip::initialize(int stage)
{
    BrokerBaseApp3::initialize(stage);
    if (stage == INITSTAGE_LOCAL) {
        int rc = fognet_create(&ctx, (int)par("hipDevice"));
        if (rc != FOGNET_OK)
            throw cRuntimeError("fognet_create: %s", fognet_status_string(rc));
    }
}

BrokerBaseAppHip::~BrokerBaseAppHip()
{
    fognet_destroy(ctx);
}

void BrokerBaseAppHip::handleMessageWhenUp(cMessage *msg)
{
    // a publish leaves the view as it is; anything else may change it
    if (dynamic_cast<MqttMsgPublish *>(msg) == nullptr)
        cacheValid = false;
    BrokerBaseApp3::handleMessageWhenUp(msg);
}

// BrokerBaseApp3.h:59
void BrokerBaseAppHip::sendPubAck(MqttMsgPublish *msg, L3Address ip, int port, bool status)
{
    if (status || brokers.empty()) {
        // the broker's own pool (:236-264) goes to the base class unchanged; with no node
        // registered the base class reaches its "no compute resource available" branch
        // (:304-318) -- after reading brokers[0] at :268, which this adapter cannot make defined
        BrokerBaseApp3::sendPubAck(msg, ip, port, status);
        return;
    }
    int32_t k = 0;
    if (cacheValid) {
        k = cachedNode;
    }
    else {
        const int32_t n = (int32_t)brokers.size();
        viewBusy.resize(n);
        viewMips.resize(n);
        bool integral = true;
        for (int32_t j = 0; j < n; ++j) {
            viewBusy[j] = brokers[j]->getBusyTime();
            viewMips[j] = brokers[j]->getMips();
            const double b = viewBusy[j];
            integral = integral && std::isfinite(b) && std::fabs(b) < 4503599627370496.0 && b == std::floor(b);
        }
        // :267-281 on the device: the same fp64 arithmetic, ties -> the lowest index
        int rc = fognet_decide(ctx, FOGNET_POLICY_REF_V3, n, viewBusy.data(), viewMips.data(),
                               msg->getMIPSRequired(), &k);
        ++decideCalls;
        if (rc == FOGNET_ERR_DIV0)  // the reference divides by node 0's MIPS (SIGFPE)
            throw cRuntimeError("BrokerBaseAppHip: node 0 has not advertised its MIPS yet");
        if (rc != FOGNET_OK)
            throw cRuntimeError("fognet_decide: %s", fognet_last_error(ctx));
        // reuse the decision for the publishes that see this view, where that is exact
        cacheValid = integral;
        cachedNode = k;
    }
    offload(msg, ip, port, k);
}

void BrokerBaseAppHip::offload(MqttMsgPublish *msg, L3Address ip, int port, int32_t k)
{
    std::ostringstream str;
    str << "request " << msg->getMIPSRequired() << " for " << msg->getRequiredTime() << " sec from "
        << brokers[k]->getBrokerId();
    FognetMsgTask *tsk = new FognetMsgTask(str.str().c_str());
    tsk->setByteLength(msg->getByteLength());
    // the request is kept with its deadline (now + requiredTime, a double)
    Request *req = new Request(msg->getClientID(), msg->getMessageID(), ip, port, msg->getMIPSRequired(),
                               simTime().dbl() + msg->getRequiredTime(), false);
    req->setRequestId(msg->getMessageID());
    requests.push_back(req);
    tsk->setRequiredMIPS(msg->getMIPSRequired());
    tsk->setRequiredTime(msg->getRequiredTime());
    tsk->setRequestID(msg->getMessageID());
    const std::string id = std::to_string(getId());
    tsk->setClientID(id.c_str());
    socket.sendTo(tsk, brokers[k]->getBrokerIp(), brokers[k]->getBrokerPort());
}

}  // namespace inet
