// TEST INFRASTRUCTURE ONLY: UDPDataIndication is declared in the stub
// (../../../../omnetpp_inet_stub.h), source address only.
#pragma once
#include "../../../../omnetpp_inet_stub.h"
