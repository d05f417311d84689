// BrokerBaseAppRec — the OMNeT++-side trace exporter: FogNetSim++'s v3 broker
// (BrokerBaseApp3, src/mqttapp/BrokerBaseApp3.{h,cc}) unchanged, plus a
// recorder of exactly the inputs the offload-decision path consumes, written
// at finish() as a FOGNTRC1 trace (include/fognet_io.h, fognet_trace_write).
// The same file then feeds libfognet_hip (fognet_run_batch, the driver
// fognetsimpp_amd/fognet_replay) and the CPU oracle: identical inputs on both
// paths.  Host code only: no device is touched.
//
// What it records, and where the reference produces it:
//   node j (CONNECT order, BrokerBaseApp3.cc:99-121: brokers[j])
//     mips     the MIPS of its first advert (FognetMsgAdvertiseMIPS.MIPS, :123-130;
//              constant in ComputeBrokerApp3, :205-222)
//     init     the tick its first advert reached the broker
//     ul       advert arrival - advert creation (the node creates the advert
//              when it sends it, ComputeBrokerApp3.cc:205-222)
//     dl       creation of the node's first status-4/5 ack (sent when the task
//              arrives, ComputeBrokerApp3.cc:282-313) - the tick the broker
//              decided that task (the publish's arrival, :138-158); a node that
//              never acked a task gets dl = ul (no task ever used it)
//   publish i (QoS 1 only, the ones the broker allocates, :138-151)
//     arrive   the tick it reached the broker;  req  its MIPSRequired
#ifndef BROKERBASEAPPREC_H
#define BROKERBASEAPPREC_H

#include <map>
#include <string>
#include <vector>

#include "inet/applications/mqttapp/BrokerBaseApp3.h"
#include "fognet_hip.h"

namespace inet {

class BrokerBaseAppRec : public BrokerBaseApp3
{
  protected:
    std::string traceFile;             // par("traceFile"): "" records nothing
    std::vector<int64_t> recArrive;    // QoS-1 publishes, broker arrival ticks (trace order)
    std::vector<int32_t> recReq;       // their MIPSRequired
    std::map<std::string, int64_t> recPublishTick;  // messageID -> decision tick (for dl)
    std::vector<int32_t> nodeMips;     // per node j (brokers[j]); 0: no advert yet
    std::vector<int64_t> nodeInit, nodeUl, nodeDl;  // -1: not observed yet

    virtual void initialize(int stage) override;
    virtual void handleMessageWhenUp(cMessage *msg) override;
    virtual void finish() override;
    // the node that sent a datagram (its control info's source address), -1 if none
    virtual int nodeOf(cMessage *msg) const;
    virtual void record(cMessage *msg);

  public:
    // the recorded inputs as fognet_batch_in (R = 1, node parameters shared); the vectors stay owned here
    fognet_batch_in recordedBatch(std::vector<int64_t> &dl, std::vector<int64_t> &ul, std::vector<int64_t> &init,
                                  std::vector<int32_t> &mips);
    int writeTrace(const char *path);  // fognet_status (FOGNET_OK, or the writer's error)
};

}  // namespace inet

#endif
