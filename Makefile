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
build/rp_attention.o: EXTRA := -fno-honor-nans

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
