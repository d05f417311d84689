// TEST INFRASTRUCTURE ONLY: the generated FognetMsgTask class
// (src/mqttapp/fognetMessages/FognetMsgTask.msg: string requestID, double
// requiredTime, string clientID, int requiredMIPS), accessors only.
#pragma once
#include "../../../../omnetpp_inet_stub.h"

namespace inet {

class FognetMsgTask : public cPacket {
    std::string requestID, clientID;
    double requiredTime = 0.0;
    int requiredMIPS = 0;
  public:
    explicit FognetMsgTask(const char *n = nullptr) : cPacket(n) {}
    const char *getRequestID() const { return requestID.c_str(); }
    void setRequestID(const char *s) { requestID = s; }
    double getRequiredTime() const { return requiredTime; }
    void setRequiredTime(double t) { requiredTime = t; }
    const char *getClientID() const { return clientID.c_str(); }
    void setClientID(const char *s) { clientID = s; }
    int getRequiredMIPS() const { return requiredMIPS; }
    void setRequiredMIPS(int m) { requiredMIPS = m; }
};

}  // namespace inet
