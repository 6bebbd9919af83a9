# Top-level build: the gfx950 HIP library (the product), the host library + CLIs above it, and
# the oracle (test infrastructure).  hipcc cross-compiles for gfx950 without a GPU present.
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
LIBDIR   := imageencoder_amd/lib
CSRC     := imageencoder_amd/csrc
OBJDIR   := build
# -ffp-contract=off: the exact FP64 path must not be fused into FMAs (reference op order);
# the FP32 fast path uses explicit fmaf and is unaffected.
HIPFLAGS := --offload-arch=$(ARCH) -mcode-object-version=5 -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -ffp-contract=off \
            -Wall -Wno-unused-function
KERNELS  := ie_encode ie_huffman ie_decode ie_pframe
OBJS     := $(addprefix $(OBJDIR)/,$(addsuffix .o,$(KERNELS) ie_capi))

.PHONY: all lib oracle ref host clean asmcheck
all: lib host oracle

lib: $(LIBDIR)/libie_hip.so

$(OBJDIR)/%.o: $(CSRC)/%.hip $(CSRC)/ie_device.h $(CSRC)/ie_common.hpp $(CSRC)/ie_dct.h $(CSRC)/ie_recbits.h include/ie_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/ie_capi.o: $(CSRC)/ie_capi.cpp $(CSRC)/ie_device.h include/ie_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libie_hip.so: $(OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

# ---- host library mirroring the reference interface (libie_host.so) + encoder/decoder CLIs
HOSTSRC   := $(wildcard $(CSRC)/host/*.cpp)
HOSTHDR   := $(wildcard $(CSRC)/host/*.hpp) include/ie_host.hpp include/ie_hip.h
HOSTFLAGS := -O2 -std=c++17 -fPIC -fopenmp -Iinclude -I$(CSRC)/host -Wall -Wextra -Wno-unused-parameter
HOSTOBJS  := $(patsubst $(CSRC)/host/%.cpp,$(OBJDIR)/host/%.o,$(HOSTSRC))
RPATH     := -Wl,-rpath,'$$ORIGIN'
host: $(LIBDIR)/libie_host.so $(LIBDIR)/encoder $(LIBDIR)/encoder_nohuff $(LIBDIR)/decoder

$(OBJDIR)/host/%.o: $(CSRC)/host/%.cpp $(HOSTHDR)
	@mkdir -p $(OBJDIR)/host
	$(CXX) $(HOSTFLAGS) -c $< -o $@

$(LIBDIR)/libie_host.so: $(HOSTOBJS) $(LIBDIR)/libie_hip.so
	$(CXX) -shared -fopenmp $(HOSTOBJS) -L$(LIBDIR) -lie_hip $(RPATH) -o $@

$(LIBDIR)/encoder: $(CSRC)/cli/main.cpp $(LIBDIR)/libie_host.so
	$(CXX) $(HOSTFLAGS) -DENCODER -DENABLE_HUFFMAN $< -L$(LIBDIR) -lie_host -lie_hip $(RPATH) -o $@
$(LIBDIR)/encoder_nohuff: $(CSRC)/cli/main.cpp $(LIBDIR)/libie_host.so
	$(CXX) $(HOSTFLAGS) -DENCODER $< -L$(LIBDIR) -lie_host -lie_hip $(RPATH) -o $@
$(LIBDIR)/decoder: $(CSRC)/cli/main.cpp $(LIBDIR)/libie_host.so
	$(CXX) $(HOSTFLAGS) -DDECODER $< -L$(LIBDIR) -lie_host -lie_hip $(RPATH) -o $@

oracle:
	$(MAKE) -C oracle oracle

ref:
	$(MAKE) -C oracle ref

# Check the exact FP64 paths really are unfused: dump the gfx950 ISA of the
# encode, decode and P-frame kernels and scan it (tools/asmcheck.py; also reports VGPRs / scratch).
ASMS := $(OBJDIR)/asm/ie_encode.s $(OBJDIR)/asm/ie_decode.s $(OBJDIR)/asm/ie_pframe.s
$(OBJDIR)/asm/%.s: $(CSRC)/%.hip $(CSRC)/ie_device.h $(CSRC)/ie_common.hpp $(CSRC)/ie_dct.h $(CSRC)/ie_recbits.h
	@mkdir -p $(OBJDIR)/asm
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o $@
asmcheck: $(ASMS)
	python3 tools/asmcheck.py $(ASMS) $(wildcard $(CSRC)/*.hip $(CSRC)/*.h $(CSRC)/*.hpp)

clean:
	rm -rf $(OBJDIR) $(LIBDIR)
