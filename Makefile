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
# bwd 310.8 -> 305.1 us at p = 0.1)
build/rp_attention.o: EXTRA := -fno-honor-nans -fno-slp-vectorize

all: $(LIB)

build/%.o: $(CSRC)/%.hip $(CSRC)/rp_common.h include/rp_api.h
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) $(EXTRA) -c $< -o $@

$(LIB): $(OBJ)
	@mkdir -p $(dir $(LIB))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJ) -o $@

clean:
	rm -rf build $(LIB)

.PHONY: all clean
