// TEST INFRASTRUCTURE ONLY: the generated message class is declared in the stub
// (../../../../omnetpp_inet_stub.h), accessors only.
#pragma once
#include "../../../../omnetpp_inet_stub.h"
