// BrokerBaseAppRec.cc — see BrokerBaseAppRec.h and INTEGRATION.md §2.
// Link: -L<repo>/fognetsimpp_amd -lfognet_hip (fognet_trace_write is host code in the library).
#include "BrokerBaseAppRec.h"

#include <cstring>

#include "fognet_io.h"
#include "inet/applications/mqttapp/fognetMessages/FognetMsgAdvertiseMIPS_m.h"
#include "inet/applications/mqttapp/mqttMessages/MqttMsgPuback_m.h"
#include "inet/transportlayer/contract/udp/UDPControlInfo_m.h"

namespace inet {

Define_Module(BrokerBaseAppRec);

void BrokerBaseAppRec::initialize(int stage)
{
    BrokerBaseApp3::initialize(stage);
    if (stage == INITSTAGE_LOCAL)
        traceFile = par("traceFile").stringValue();
}

void BrokerBaseAppRec::handleMessageWhenUp(cMessage *msg)
{
    // before the base class: it removes the control info and deletes the message
    if (!traceFile.empty())
        record(msg);
    BrokerBaseApp3::handleMessageWhenUp(msg);
}

int BrokerBaseAppRec::nodeOf(cMessage *msg) const
{
    const UDPDataIndication *ctrl = dynamic_cast<const UDPDataIndication *>(msg->getControlInfo());
    if (!ctrl)
        return -1;
    for (unsigned int j = 0; j < brokers.size(); j++)
        if (brokers[j]->getBrokerIp() == ctrl->getSrcAddr())
            return (int)j;
    return -1;
}

void BrokerBaseAppRec::record(cMessage *msg)
{
    if (msg->isSelfMessage())
        return;
    const int64_t now = simTime().raw();
    if (MqttMsgPublish *p = dynamic_cast<MqttMsgPublish *>(msg)) {
        if (p->getQoS() == 1) {  // the publishes the broker allocates (BrokerBaseApp3.cc:138-151)
            recArrive.push_back(now);
            recReq.push_back(p->getMIPSRequired());
            recPublishTick[p->getMessageID()] = now;
        }
        return;
    }
    if (nodeMips.size() < brokers.size()) {  // nodes registered since (CONNECT order, :99-121)
        nodeMips.resize(brokers.size(), 0);
        nodeInit.resize(brokers.size(), -1);
        nodeUl.resize(brokers.size(), -1);
        nodeDl.resize(brokers.size(), -1);
    }
    if (FognetMsgAdvertiseMIPS *a = dynamic_cast<FognetMsgAdvertiseMIPS *>(msg)) {
        // the node matched by id, as the view update does (:123-130); its first advert only
        for (unsigned int j = 0; j < brokers.size(); j++)
            if (strcmp(brokers[j]->getBrokerId(), a->getComputeBrokerID()) == 0 && nodeInit[j] < 0) {
                nodeMips[j] = a->getMIPS();
                nodeInit[j] = now;
                nodeUl[j] = now - a->getCreationTime().raw();
            }
        return;
    }
    if (MqttMsgPuback *ack = dynamic_cast<MqttMsgPuback *>(msg)) {
        // status 5 (assigned) / 4 (queued): created when the task reached the node
        if (ack->getStatus() != 4 && ack->getStatus() != 5)
            return;
        const int j = nodeOf(msg);
        if (j < 0 || nodeDl[j] >= 0)
            return;
        std::map<std::string, int64_t>::const_iterator it = recPublishTick.find(ack->getMessageID());
        if (it != recPublishTick.end())
            nodeDl[j] = ack->getCreationTime().raw() - it->second;
    }
}

fognet_batch_in BrokerBaseAppRec::recordedBatch(std::vector<int64_t> &dl, std::vector<int64_t> &ul,
                                                std::vector<int64_t> &init, std::vector<int32_t> &mips)
{
    const size_t n = brokers.size();
    dl.assign(n, 0);
    ul.assign(n, 0);
    init.assign(n, 0);
    mips.assign(n, 0);
    for (size_t j = 0; j < n && j < nodeMips.size(); j++) {
        mips[j] = nodeMips[j];
        init[j] = nodeInit[j] < 0 ? 0 : nodeInit[j];
        ul[j] = nodeUl[j] < 0 ? 0 : nodeUl[j];
        dl[j] = nodeDl[j] < 0 ? ul[j] : nodeDl[j];  // never acked a task: no replay reads it
    }
    fognet_batch_in in;
    memset(&in, 0, sizeof in);
    in.R = 1;
    in.T = (int32_t)recArrive.size();
    in.N = (int32_t)n;
    in.node_stride = 0;
    in.policy = FOGNET_POLICY_REF_V3;
    in.arrive_tick = recArrive.data();
    in.req_mips = recReq.data();
    in.mips = mips.data();
    in.dl_tick = dl.data();
    in.ul_tick = ul.data();
    in.init_adv_tick = init.data();
    return in;
}

int BrokerBaseAppRec::writeTrace(const char *path)
{
    std::vector<int64_t> dl, ul, init;
    std::vector<int32_t> mips;
    const fognet_batch_in in = recordedBatch(dl, ul, init, mips);
    const std::string note = "recorded by BrokerBaseAppRec at " + getFullPath();
    return fognet_trace_write(path, &in, nullptr, note.c_str());
}

void BrokerBaseAppRec::finish()
{
    if (!traceFile.empty()) {
        const int rc = writeTrace(traceFile.c_str());
        if (rc != FOGNET_OK)
            throw cRuntimeError("BrokerBaseAppRec: writing %s: %s", traceFile.c_str(), fognet_io_last_error());
    }
    BrokerBaseApp3::finish();
}

}  // namespace inet
