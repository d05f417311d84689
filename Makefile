# libfognet_hip: gfx950 kernels + C ABI.  hipcc cross-compiles without a GPU.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC -Wall -Wno-unused-result
SRC_DIR := fognetsimpp_amd/csrc
SRCS := $(SRC_DIR)/capi.hip $(SRC_DIR)/replay.hip $(SRC_DIR)/replay_wide.hip $(SRC_DIR)/replay_v2.hip $(SRC_DIR)/replay_region.hip $(SRC_DIR)/decide.hip $(SRC_DIR)/tracegen.hip $(SRC_DIR)/user_stats.hip
HDRS := include/fognet_hip.h include/fognet_io.h $(SRC_DIR)/internal.h $(SRC_DIR)/replay_common.h
OBJDIR := build/obj
OBJS := $(patsubst $(SRC_DIR)/%.hip,$(OBJDIR)/%.o,$(SRCS)) $(OBJDIR)/io.o
HOSTCXX ?= g++
LIB := fognetsimpp_amd/libfognet_hip.so

DRIVER := fognetsimpp_amd/fognet_replay

all: $(LIB) $(DRIVER) oracle

# command-line trace-replay driver (host C++ over the C ABI; reads omnetpp.ini keys)
$(DRIVER): $(SRC_DIR)/fognet_replay.cpp include/fognet_hip.h include/fognet_io.h $(LIB)
	$(HOSTCXX) -O2 -std=c++17 -Wall -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ $< -o $@ \
	  -Lfognetsimpp_amd -lfognet_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib

$(OBJDIR)/%.o: $(SRC_DIR)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@

$(OBJDIR)/io.o: $(SRC_DIR)/io.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HOSTCXX) -O2 -std=c++17 -fPIC -Wall -ffp-contract=off -Iinclude -c $< -o $@

# replay.o keeps its gfx950 assembly: the inline-asm prefetch of replay.hip is
# correct only while no compiler-generated instruction of the replay loops
# touches the reserved registers, so the library is not linked
# unless tools/check_nh_regs.py passes on exactly the code that ships.
$(OBJDIR)/replay.o: $(SRC_DIR)/replay.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o $@ -save-temps=obj
	python3 tools/check_nh_regs.py $(OBJDIR)/replay-hip-amdgcn-amd-amdhsa-$(ARCH).s

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C oracle

asm: $(SRC_DIR)/replay.hip $(HDRS)
	@mkdir -p build/asm
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -Iinclude -c $< -o build/asm/replay.o -save-temps=obj -Rpass-analysis=kernel-resource-usage

clean:
	rm -rf build $(LIB) $(DRIVER)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean asm

# Profile build: replay_kernel writes loop counters into the stats record
# (tools/replay_counters.py); not used by the product path.
PROF_LIB := build/prof/libfognet_hip.so
prof: $(SRCS) $(HDRS)
	@mkdir -p build/prof
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DFOGNET_REPLAY_PROFILE=1 -Iinclude -shared -o $(PROF_LIB) $(SRCS) $(SRC_DIR)/io.cpp
	@mkdir -p build/prof2
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DFOGNET_REPLAY_PROFILE=2 -Iinclude -shared -o build/prof2/libfognet_hip.so $(SRCS) $(SRC_DIR)/io.cpp

.PHONY: prof

# Host code under AddressSanitizer + UBSan: the CPU oracle, the
# trace / result-file I/O and the command-line driver, each driven through its
# paths by a standalone program (no Python, no GPU: the driver runs --dry-run
# and its error paths).  `make asan` builds and runs them; any report fails it.
ASAN_FLAGS := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1
ASAN_DIR := build/asan
asan:
	@mkdir -p $(ASAN_DIR)
	gcc $(ASAN_FLAGS) -std=gnu11 -ffp-contract=off -pthread tests/c/oracle_check.c oracle/fognet_oracle.c \
	  oracle/fognet_oracle_v2.c -lm -o $(ASAN_DIR)/oracle_check
	$(HOSTCXX) $(ASAN_FLAGS) -std=c++17 -ffp-contract=off -Iinclude tests/c/io_check.cpp $(SRC_DIR)/io.cpp \
	  -o $(ASAN_DIR)/io_check
	$(HOSTCXX) $(ASAN_FLAGS) -std=c++17 -ffp-contract=off -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
	  $(SRC_DIR)/fognet_replay.cpp $(SRC_DIR)/io.cpp -o $(ASAN_DIR)/fognet_replay \
	  -Lfognetsimpp_amd -lfognet_hip -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$(CURDIR)/fognetsimpp_amd -Wl,-rpath,/opt/rocm/lib
	ASAN_OPTIONS=detect_leaks=1 $(ASAN_DIR)/oracle_check
	ASAN_OPTIONS=detect_leaks=1 $(ASAN_DIR)/io_check $(ASAN_DIR)
	ASAN_OPTIONS=detect_leaks=0 $(ASAN_DIR)/fognet_replay -f tests/scenarios/fog5.ini --users 'user[10]' --reps 3 \
	  --dry-run --show --trace-out $(ASAN_DIR)/drv.fogntrc > /dev/null
	ASAN_OPTIONS=detect_leaks=0 $(ASAN_DIR)/fognet_replay -f tests/scenarios/fog5.ini -c Example --nodes 5 --dry-run > /dev/null
	! ASAN_OPTIONS=detect_leaks=0 $(ASAN_DIR)/fognet_replay -f tests/scenarios/fog5.ini -c Early --users 'user[2]' --dry-run 2> $(ASAN_DIR)/err.txt
	grep -q "divide by the unadvertised MIPS 0" $(ASAN_DIR)/err.txt
	! ASAN_OPTIONS=detect_leaks=0 $(ASAN_DIR)/fognet_replay -f tests/scenarios/fog5.ini --users 'user[2]' --ring 1000 --dry-run 2> $(ASAN_DIR)/err.txt
	@echo "asan: oracle, io and driver clean"

.PHONY: asan
