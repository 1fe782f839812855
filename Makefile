# Builds the MI355X HIP library behind include/rp_api.h (gfx950 only).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := repurpose_amd/csrc
SRC := $(wildcard $(CSRC)/*.hip)
OBJ := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRC))
LIB := repurpose_amd/_native/librepurpose_amd.so
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -Wall -Wno-unused-variable

# attention: no NaN semantics needed (scores are finite or -inf), drops the canonicalising
# v_max before every fmaxf of an MFMA result
# -fno-slp-vectorize: no v_pk_*_f32 packing of the softmax / row-sum VALU, which issues beside the
# MFMAs at a higher cost than the scalar pairs (MI355X attention microbench: fwd 162.6 -> 153.1 us,
# bwd 310.8 -> 305.1 us at p = 0.1).  An explicit machine-scheduler occupancy/latency bias (any of
# 0..40 measured alike; 20 kept) schedules the tile loops for latency: fwd p=0.1 160 -> 150 us,
# bwd p=0.1 310 -> 301 us, p=0 fwd 119 -> 112 us, bwd 299 -> 286 us (interleaved runs, one box)
build/rp_attention.o: EXTRA := -fno-honor-nans -fno-slp-vectorize -mllvm -amdgpu-schedule-metric-bias=20

all: $(LIB)

build/%.o: $(CSRC)/%.hip $(CSRC)/rp_common.h include/rp_api.h Makefile
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
