# Build liborleans_route.so (HIP, gfx950) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function
SRC = orleans_amd/csrc/route_kernels.hip orleans_amd/csrc/wire_codec.hip orleans_amd/csrc/orl_api.cpp orleans_amd/csrc/orl_node.cpp
HDR = include/orleans_route.h orleans_amd/csrc/orl_internal.h
LIB = orleans_amd/liborleans_route.so
OBJ = build/route_kernels.o build/wire_codec.o build/orl_api.o build/orl_node.o
# RCCL (the node exchange); inside a torch process the soname resolves to torch's loaded copy
LIBS = -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl

all: $(LIB) oracle

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) $(LIBS)

build/route_kernels.o: orleans_amd/csrc/route_kernels.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/wire_codec.o: orleans_amd/csrc/wire_codec.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

build/orl_api.o: orleans_amd/csrc/orl_api.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

build/orl_node.o: orleans_amd/csrc/orl_node.cpp $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -x hip -c -o $@ $<

oracle:
	$(MAKE) -C oracle

# A/B build of the kernels with extra defines, for the lab scripts only (LAB_LIB=lab/liborleans_route_<NAME>.so):
#   make lab NAME=fan512 DEFS=-DORL_FAN_LDS=512
lab: build/wire_codec.o build/orl_api.o build/orl_node.o
	@mkdir -p build lab
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o build/route_kernels_$(NAME).o orleans_amd/csrc/route_kernels.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -o lab/liborleans_route_$(NAME).so build/route_kernels_$(NAME).o build/wire_codec.o \
		build/orl_api.o build/orl_node.o $(LIBS)

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean lab
