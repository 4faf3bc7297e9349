# Builds dgppo_fov_amd/lib/libdgppo_hip.so for gfx950 (MI355X).  `make -j8`.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := dgppo_fov_amd/csrc
OUT := dgppo_fov_amd/lib
OBJ := dgppo_fov_amd/_build
SRCS := $(wildcard $(CSRC)/*.hip)
OBJS := $(patsubst $(CSRC)/%.hip,$(OBJ)/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.h) include/dgppo_hip.h
# env kernels must not contract a*b+c into FMA (bit parity with the NumPy oracle): env_step.hip and
# math32.h carry `#pragma clang fp contract(off)`; the network kernels keep the default (FMA).
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Iinclude

all: $(OUT)/libdgppo_hip.so

$(OBJ)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OUT)/libdgppo_hip.so: $(OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJS)

clean:
	rm -rf $(OBJ) $(OUT)/libdgppo_hip.so

.PHONY: all clean
