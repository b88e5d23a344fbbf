# Top-level build (no cmake): hipcc for gfx950, in-tree outputs.
#
#   make            libgossip_amd.so + the drop-in Application + the oracle checker
#   make lib        gossip_protocol_amd/libgossip_amd.so  (the product: HIP kernels + C ABI)
#   make app        gossip_protocol_amd/bin/Application    (Application-shaped driver on the
#                   MP1Node/EmulNet/Params/Log facade; Grader.sh-compatible)
#   make oracle     oracle/liboracle.so (+ oracle/_ref when /root/reference exists)

HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
JOBS     ?= 8
PKG      := gossip_protocol_amd
CSRC     := $(PKG)/csrc
LIB      := $(PKG)/libgossip_amd.so
APP      := $(PKG)/bin/Application
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Iinclude -I$(CSRC) \
            -I/opt/rocm/include
LDFLAGS  := -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

KERNELS  := $(wildcard $(CSRC)/*.hip)
HOSTSRC  := $(wildcard $(CSRC)/*.cpp)
OBJS     := $(patsubst $(CSRC)/%.hip,build/%.hip.o,$(KERNELS)) \
            $(patsubst $(CSRC)/%.cpp,build/%.cpp.o,$(HOSTSRC))
HDRS     := $(wildcard $(CSRC)/*.hpp) $(wildcard include/gossip/*.h) $(wildcard include/gossip/*.hpp)

.PHONY: all lib app oracle clean lib-variant pv-variant
all: lib app oracle

lib: $(LIB)
app: $(APP) $(PKG)/bin/RecvDriver

build:
	mkdir -p build

# header dependencies from the compiler (-MMD): an object rebuilds when a header it includes
# changes, not on every header edit (pview_kernels.hip alone takes minutes)
build/%.hip.o: $(CSRC)/%.hip | build
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

build/%.cpp.o: $(CSRC)/%.cpp | build
	$(HIPCC) $(HIPFLAGS) -MMD -MP -c $< -o $@

-include $(wildcard build/*.d)

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -o $@ $(OBJS) $(LDFLAGS)

$(APP): $(PKG)/app/app_main.cpp $(LIB) include/gossip/mp1_facade.hpp
	mkdir -p $(PKG)/bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ $(PKG)/app/app_main.cpp \
	    -L$(PKG) -lgossip_amd -Wl,-rpath,'$$ORIGIN/..'

# test driver of the receive-side entry points (tests/drivers/recv_driver.cpp); the same source
# is built against the reference under oracle/_ref/RecvDriver
$(PKG)/bin/RecvDriver: tests/drivers/recv_driver.cpp $(LIB) include/gossip/mp1_facade.hpp
	mkdir -p $(PKG)/bin
	g++ -O2 -std=c++17 -Wall -Iinclude -o $@ tests/drivers/recv_driver.cpp \
	    -L$(PKG) -lgossip_amd -Wl,-rpath,'$$ORIGIN/..'

oracle: lib
	$(MAKE) -C oracle

# kernel A/B variant: make lib-variant TAG=x VFLAGS=-DGSP_...  ->  $(PKG)/libgossip_amd.x.so
# (loaded with GSP_LIB_VARIANT=x; experiments only, the product is $(LIB))
lib-variant: $(KERNELS) $(HOSTSRC) $(HDRS)
	mkdir -p build/v-$(TAG)
	for f in $(KERNELS) $(HOSTSRC); do \
	  $(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $$f -o build/v-$(TAG)/$$(basename $$f).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -o $(PKG)/libgossip_amd.$(TAG).so build/v-$(TAG)/*.o $(LDFLAGS)

# partial-view kernel A/B variant, rebuilding only pview_kernels.hip (the other objects come
# from build/): make pv-variant TAG=x VFLAGS=-DGSP_...  ->  $(PKG)/libgossip_amd.x.so
pv-variant: $(OBJS)
	mkdir -p build/v-$(TAG)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $(CSRC)/pview_kernels.hip -o build/v-$(TAG)/pview_kernels.hip.o
	$(HIPCC) --offload-arch=$(ARCH) -o $(PKG)/libgossip_amd.$(TAG).so build/v-$(TAG)/pview_kernels.hip.o \
	    $(filter-out build/pview_kernels.hip.o,$(OBJS)) $(LDFLAGS)

clean:
	rm -rf build $(LIB) $(PKG)/libgossip_amd.*.so $(PKG)/bin
	$(MAKE) -C oracle clean
