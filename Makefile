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

# diagnostic library with the persistent rollout's phase timers (scripts/env_stamps.py; DGPPO_HIP_LIB points at it)
STAMP_OBJS := $(filter-out $(OBJ)/env_step.o,$(OBJS)) $(OBJ)/env_step_stamps.o
$(OBJ)/env_step_stamps.o: $(CSRC)/env_step.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DDGPPO_ENV_STAMPS -c $< -o $@
stamps: $(STAMP_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OUT)/libdgppo_hip_stamps.so $(STAMP_OBJS)

# diagnostic library with every env-graph store dropped from the wave kernels (timing experiments only)
NOSTORE_OBJS := $(filter-out $(OBJ)/env_step.o,$(OBJS)) $(OBJ)/env_step_nostore.o
$(OBJ)/env_step_nostore.o: $(CSRC)/env_step.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DDGPPO_DIAG_NOSTORE -c $< -o $@
nostore: $(NOSTORE_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OUT)/libdgppo_hip_nostore.so $(NOSTORE_OBJS)

clean:
	rm -rf $(OBJ) $(OUT)/libdgppo_hip.so

.PHONY: all clean stamps nostore

# diagnostic library with the fused policy step's phase timestamps (scripts/policy_probe.py; DGPPO_HIP_LIB points at it)
PROBE_OBJS := $(filter-out $(OBJ)/policy.o,$(OBJS)) $(OBJ)/policy_probe.o
$(OBJ)/policy_probe.o: $(CSRC)/policy.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DPOLICY_PROBE -c $< -o $@
probe: $(PROBE_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OUT)/libdgppo_hip_probe.so $(PROBE_OBJS)

# register-form policy step at 4 waves per SIMD instead of the default 3 (A/B: DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_w4.so)
W4_OBJS := $(filter-out $(OBJ)/policy.o,$(OBJS)) $(OBJ)/policy_w4.o
$(OBJ)/policy_w4.o: $(CSRC)/policy.hip $(HDRS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -DPOLICY_REG_WAVES=4 -c $< -o $@
w4: $(W4_OBJS)
	@mkdir -p $(OUT)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $(OUT)/libdgppo_hip_w4.so $(W4_OBJS)
