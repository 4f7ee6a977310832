# Builds libliteasr_hip.so (gfx950) from liteasr_amd/csrc/*.hip and the C oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH  ?= gfx950
SRC   := $(wildcard liteasr_amd/csrc/*.hip)
OBJ   := $(patsubst liteasr_amd/csrc/%.hip,build/obj/%.o,$(SRC))
LIB   := liteasr_amd/lib/libliteasr_hip.so
IOLIB := liteasr_amd/lib/libliteasr_io.so
DECLIB := liteasr_amd/lib/libliteasr_decode.so
COMMLIB := liteasr_amd/lib/libliteasr_comm.so
CXX   ?= g++
HDRS  := liteasr_amd/csrc/common.h liteasr_amd/csrc/tile.h liteasr_amd/csrc/gemm_kernel.h liteasr_amd/csrc/gemm_launch.h include/liteasr_hip.h
FLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC

all: $(LIB) $(IOLIB) $(DECLIB) $(COMMLIB)

# host-only native feature reader (no device code); -ffp-contract=off keeps the decode
# arithmetic bit-identical to the reference's numpy float32 expressions
$(IOLIB): liteasr_amd/csrc/io/ark_io.cpp include/liteasr_io.h
	@mkdir -p liteasr_amd/lib
	$(CXX) -O2 -std=c++17 -fPIC -shared -ffp-contract=off -pthread -o $@ $<

# host-only CTC prefix beam search (inference); same fp-contract rule, so its double
# arithmetic matches the reference's Python floats
$(DECLIB): liteasr_amd/csrc/decode/prefix_beam.cpp include/liteasr_decode.h
	@mkdir -p liteasr_amd/lib
	$(CXX) -O2 -std=c++17 -fPIC -shared -ffp-contract=off -o $@ $<

# host-only bucketed gradient reducer over RCCL (HIP runtime streams/events, no kernels)
$(COMMLIB): liteasr_amd/csrc/comm/reducer.cpp include/liteasr_comm.h
	@mkdir -p liteasr_amd/lib
	$(HIPCC) -O2 -std=c++17 -fPIC -shared -o $@ $< -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

build/obj/%.o: liteasr_amd/csrc/%.hip $(HDRS)
	@mkdir -p build/obj
	$(HIPCC) $(FLAGS) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p liteasr_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $^

clean:
	rm -rf build $(LIB) $(IOLIB) $(DECLIB) $(COMMLIB)

.PHONY: all clean
