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

# Host-side sanitizer build of the C ABI: the launchers' argument validation,
# workspace queries and host arithmetic compiled with AddressSanitizer + UndefinedBehaviorSanitizer
# (host code only: -Xarch_host; the device code is compiled as usual), driven through every error path by
# tests/native/abi_errors.cpp.  Runs without a GPU; tests/test_asan_abi.py runs it.
ASAN_DIR := build/asan
ASAN_FLAGS := -O1 -g -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -fno-omit-frame-pointer \
	-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all
ASAN_OBJ := $(patsubst $(CSRC)/%.hip,$(ASAN_DIR)/%.o,$(SRC))

$(ASAN_DIR)/%.o: $(CSRC)/%.hip $(CSRC)/rp_common.h include/rp_api.h Makefile
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(ASAN_FLAGS) -c $< -o $@

$(ASAN_DIR)/abi_errors: tests/native/abi_errors.cpp $(ASAN_OBJ) include/rp_api.h
	$(HIPCC) -x c++ -O1 -g -std=c++17 -Iinclude -fno-omit-frame-pointer -fsanitize=address,undefined \
		-fno-sanitize-recover=all -c tests/native/abi_errors.cpp -o $(ASAN_DIR)/abi_errors.o
	$(HIPCC) -fsanitize=address,undefined $(ASAN_DIR)/abi_errors.o $(ASAN_OBJ) -o $@

asan: $(ASAN_DIR)/abi_errors

.PHONY: asan
