// TEST INFRASTRUCTURE ONLY: the few OMNeT++ 4.6 / INET 3.3 identifiers that
// integration/BrokerBaseAppHip.{h,cc} touches, declared with the signatures the
// reference's headers and generated message classes give them
// (src/mqttapp/BrokerBaseApp3.h:24-64, Broker.cc, Request.cc, the .msg files),
// so the adapter can be type-checked (-fsyntax-only) and driven on a GPU
// (tests/adapter/adapter_drive.cpp) where OMNeT++ is absent.  Not a build of
// the reference: no reference source is compiled against this.
#pragma once
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace inet {

typedef int64_t int64;

struct SimTime {
    int64 raw_ = 0;  // 1e-12 s
    double dbl() const { return (double)raw_ * 1e-12; }
    int64 raw() const { return raw_; }
};
SimTime simTime();  // the driver's clock

class cRuntimeError : public std::runtime_error {
    static std::string fmt(const char *f, va_list ap) {
        char buf[512];
        vsnprintf(buf, sizeof buf, f, ap);
        return buf;
    }
  public:
    cRuntimeError(const char *f, ...) : std::runtime_error(f) {
        va_list ap;
        va_start(ap, f);
        static_cast<std::runtime_error&>(*this) = std::runtime_error(fmt(f, ap));
        va_end(ap);
    }
};

class cObject {
  public:
    virtual ~cObject() {}
};

class cMessage : public cObject {
    std::string name;
    SimTime created = simTime();
    cObject *ctrl = nullptr;
    short kind = 0;
  public:
    explicit cMessage(const char *n = nullptr) : name(n ? n : "") {}
    virtual ~cMessage() { delete ctrl; }
    const char *getName() const { return name.c_str(); }
    SimTime getCreationTime() const { return created; }
    cObject *getControlInfo() const { return ctrl; }
    void setControlInfo(cObject *c) { ctrl = c; }
    bool isSelfMessage() const { return false; }
    short getKind() const { return kind; }
    void setKind(short k) { kind = k; }
    void stubSetCreationTime(int64 t) { created.raw_ = t; }  // stub only: the driver's sender clock
};

class cPacket : public cMessage {
    int64 byteLength = 0;
  public:
    explicit cPacket(const char *n = nullptr) : cMessage(n) {}
    int64 getByteLength() const { return byteLength; }
    void setByteLength(int64 l) { byteLength = l; }
};

class L3Address {
    uint32_t a = 0;
  public:
    L3Address() {}
    explicit L3Address(uint32_t x) : a(x) {}
    uint32_t raw() const { return a; }
};

// INET 3.3 UDPDataIndication (the control info of a received datagram)
class UDPDataIndication : public cObject {
    L3Address src;
  public:
    explicit UDPDataIndication(L3Address a) : src(a) {}
    L3Address getSrcAddr() const { return src; }
};
inline bool operator==(const L3Address &a, const L3Address &b) { return a.raw() == b.raw(); }

class UDPSocket {
  public:
    void sendTo(cPacket *msg, L3Address destAddr, int destPort);  // the driver's network
};

class cPar {
    long v = 0;
    std::string str;
  public:
    explicit cPar(long x = 0) : v(x) {}
    operator int() const { return (int)v; }
    operator long() const { return v; }
    const char *stringValue() const { return str.c_str(); }
    void stubSet(const std::string &x) { str = x; }
};

enum { INITSTAGE_LOCAL = 0, NUM_INIT_STAGES = 12 };

class ApplicationBase {
  protected:
    cPar parHipDevice, parTraceFile;
    virtual void initialize(int stage) {}
    virtual void handleMessageWhenUp(cMessage *msg) = 0;
    virtual void finish() {}
  public:
    virtual ~ApplicationBase() {}
    cPar &par(const char *name) { return std::string(name) == "traceFile" ? parTraceFile : parHipDevice; }
    int getId() const { return 7; }
    std::string getFullPath() const { return "FogNet.broker.udpApp[0]"; }
};

// generated message classes (opp_string fields: const char * getters/setters)
class MqttMsgPublish : public cPacket {
    std::string clientID, messageID;
    int qoS = 1, MIPSRequired = 0;
    double requiredTime = 0.0;
  public:
    explicit MqttMsgPublish(const char *n = nullptr) : cPacket(n) {}
    const char *getClientID() const { return clientID.c_str(); }
    void setClientID(const char *s) { clientID = s; }
    const char *getMessageID() const { return messageID.c_str(); }
    void setMessageID(const char *s) { messageID = s; }
    int getQoS() const { return qoS; }
    void setQoS(int q) { qoS = q; }
    int getMIPSRequired() const { return MIPSRequired; }
    void setMIPSRequired(int m) { MIPSRequired = m; }
    double getRequiredTime() const { return requiredTime; }
    void setRequiredTime(double t) { requiredTime = t; }
};

// src/mqttapp/mqttMessages/MqttMsgPuback.msg: the acks a node sends (status 4 queued, 5 assigned,
// 6 performed) and the broker relays (BrokerBaseApp3.cc:164-198)
class MqttMsgPuback : public cPacket {
    std::string messageID;
    int status = 0;
  public:
    explicit MqttMsgPuback(const char *n = nullptr) : cPacket(n) {}
    const char *getMessageID() const { return messageID.c_str(); }
    void setMessageID(const char *s) { messageID = s; }
    int getStatus() const { return status; }
    void setStatus(int x) { status = x; }
};

class FognetMsgAdvertiseMIPS : public cPacket {
    int MIPS = 0;
    std::string computeBrokerID;
    double busyTime = 0.0;
  public:
    explicit FognetMsgAdvertiseMIPS(const char *n = nullptr) : cPacket(n) {}
    int getMIPS() const { return MIPS; }
    void setMIPS(int m) { MIPS = m; }
    const char *getComputeBrokerID() const { return computeBrokerID.c_str(); }
    void setComputeBrokerID(const char *s) { computeBrokerID = s; }
    double getBusyTime() const { return busyTime; }
    void setBusyTime(double b) { busyTime = b; }
};

// src/mqttapp/Broker.cc: the broker's record of one compute broker (fog node)
class Broker {
    const char *brokerID = nullptr;
    L3Address brokerIP;
    int brokerPort = 0;
    int MIPS = 0;
    double busyTime = 0.0;
  public:
    Broker(const char *id, L3Address ip, int port, int mips) : brokerID(id), brokerIP(ip), brokerPort(port), MIPS(mips) {}
    const char *getBrokerId() const { return brokerID; }
    const L3Address &getBrokerIp() const { return brokerIP; }
    int getBrokerPort() const { return brokerPort; }
    int getMips() const { return MIPS; }
    void setMips(int m) { MIPS = m; }
    double getBusyTime() const { return busyTime; }
    void setBusyTime(double b) { busyTime = b; }
};

// src/mqttapp/Request.cc
class Request {
    const char *clientID, *requestID;
    L3Address clientIP;
    int clientPort, requiredMIPS;
    double requiredTime;
    bool status;
  public:
    Request(const char *c, const char *r, L3Address ip, int port, int mips, double t, bool st)
        : clientID(c), requestID(r), clientIP(ip), clientPort(port), requiredMIPS(mips), requiredTime(t), status(st) {}
    void setRequestId(const char *r) { requestID = r; }
    double getRequiredTime() const { return requiredTime; }
};

#define Define_Module(CLASS) static int define_module_##CLASS __attribute__((unused)) = 0

}  // namespace inet
