# Top-level build: the product library (HIP for gfx950) and the test oracle.
#
#   make            -> voxelraytrace20190722_amd/libvrt.so + oracle/liboracle.so
#                      (+ oracle/_ref/libvrtref.so when /root/reference exists)
#
# Float contract: -ffp-contract=off (no FMA contraction, host or device), no
# fast-math; hipcc keeps correctly rounded f32 division and sqrt by default.

HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
PKG := voxelraytrace20190722_amd
SRC := $(PKG)/csrc
BLD := build/obj
FP := -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt
HIPFLAGS := -x hip --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 $(FP) -Iinclude -I$(SRC) \
            -Wall -Wno-unused-function -fvisibility=hidden
CXXFLAGS := -O2 -fPIC -std=c++17 -ffp-contract=off -Iinclude -Wall -fvisibility=hidden

LIBS := -L/opt/rocm/lib -lrccl -lpthread
HOSTOBJS := $(BLD)/vrt_host.o $(BLD)/vrt_legacy.o $(BLD)/vrt_multi.o $(BLD)/vrt_hdr.o $(BLD)/vrt_proxy.o $(BLD)/vrt_obj.o $(BLD)/vrt_tga.o
OBJS := $(BLD)/vrt_kernels.o $(BLD)/vrt_build.o $(HOSTOBJS) $(BLD)/vrt_build_id.o
HDRS := include/vrt.h $(SRC)/vrt_math.h $(SRC)/vrt_internal.h $(SRC)/vrt_error.h

all: $(PKG)/libvrt.so oracle

$(BLD):
	mkdir -p $(BLD)

# wave-level atomic aggregation by a DPP scan (the default iterative scan
# loops over the active lanes; take_unit() adds a lane-varying value)
KFLAGS := -mllvm -amdgpu-atomic-optimizer-strategy=DPP

$(BLD)/vrt_kernels.o: $(SRC)/vrt_kernels.hip $(HDRS) | $(BLD)
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) -c $< -o $@

$(BLD)/vrt_build.o: $(SRC)/vrt_build.hip $(HDRS) | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BLD)/vrt_host.o: $(SRC)/vrt_host.cpp $(HDRS) | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the reference's primitives under their C++ (mangled) names; must not see
# vrt.h's extern "C" declarations of the same signatures
$(BLD)/vrt_legacy.o: $(SRC)/vrt_legacy.cpp $(SRC)/vrt_math.h | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the multi-device frame: RCCL (ncclCommInitAll + ncclGather over xGMI)
$(BLD)/vrt_multi.o: $(SRC)/vrt_multi.cpp $(HDRS) | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BLD)/vrt_hdr.o: $(SRC)/vrt_hdr.cpp include/vrt.h | $(BLD)
	g++ $(CXXFLAGS) -c $< -o $@

$(BLD)/vrt_proxy.o: $(SRC)/vrt_proxy.cpp include/vrt.h | $(BLD)
	g++ $(CXXFLAGS) -c $< -o $@

$(BLD)/vrt_obj.o: $(SRC)/vrt_obj.cpp include/vrt.h $(SRC)/vrt_error.h | $(BLD)
	g++ $(CXXFLAGS) -c $< -o $@

$(BLD)/vrt_tga.o: $(SRC)/vrt_tga.cpp include/vrt.h $(SRC)/vrt_error.h | $(BLD)
	g++ $(CXXFLAGS) -c $< -o $@

# vrt_build_id(): the source hash (tools/build_id.py); the C file is
# rewritten only when the hash changes
$(BLD)/vrt_build_id.c: FORCE | $(BLD)
	python3 tools/build_id.py --write $@

$(BLD)/vrt_build_id.o: $(BLD)/vrt_build_id.c
	gcc -O2 -fPIC -c $< -o $@

FORCE:

$(PKG)/libvrt.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) $(LIBS)

oracle:
	$(MAKE) -C oracle

# A/B variant of the kernels:  make variant NAME=v0 DEFS="-DVRT_EXPAND_V=0"
variant: $(HOSTOBJS) $(BLD)/vrt_build.o | $(BLD)
	mkdir -p build/ab
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) $(DEFS) -c $(SRC)/vrt_kernels.hip -o build/ab/k_$(NAME).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/ab/libvrt_$(NAME).so \
	  build/ab/k_$(NAME).o $(BLD)/vrt_build.o $(HOSTOBJS) $(BLD)/vrt_build_id.o $(LIBS)

# variant that also rebuilds the host side (for data-layout changes)
fullvariant: $(BLD)/vrt_build.o $(BLD)/vrt_legacy.o $(BLD)/vrt_multi.o $(BLD)/vrt_hdr.o $(BLD)/vrt_proxy.o $(BLD)/vrt_obj.o $(BLD)/vrt_tga.o | $(BLD)
	mkdir -p build/ab
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) $(DEFS) -c $(SRC)/vrt_kernels.hip -o build/ab/k_$(NAME).o
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c $(SRC)/vrt_host.cpp -o build/ab/h_$(NAME).o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o build/ab/libvrt_$(NAME).so \
	  build/ab/k_$(NAME).o build/ab/h_$(NAME).o $(BLD)/vrt_build.o $(BLD)/vrt_legacy.o $(BLD)/vrt_multi.o \
	  $(BLD)/vrt_hdr.o $(BLD)/vrt_proxy.o $(BLD)/vrt_obj.o $(BLD)/vrt_tga.o $(BLD)/vrt_build_id.o $(LIBS)

# ISA listing + register/occupancy report of the kernels (for DESIGN.md)
isa: | $(BLD)
	$(HIPCC) $(HIPFLAGS) $(KFLAGS) --offload-device-only -S $(SRC)/vrt_kernels.hip -o $(BLD)/vrt_kernels.s \
	  -Rpass-analysis=kernel-resource-usage 2> $(BLD)/resource_usage.txt || true

clean:
	rm -rf build $(PKG)/libvrt.so
	$(MAKE) -C oracle clean

.PHONY: all oracle isa clean FORCE
