# Builds the gfx950 HIP library behind the C ABI in include/sv_ge2e.h, plus its fault-injection
# test build (libsv_ge2e_faultinj.so: the same sources with -DSV_FAULT_INJECTION, which exports
# sv_test_set_fault; only tests/test_gpu_status.py loads it).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
PKG := pytorch_speaker_verification_amd
SRC := $(wildcard $(PKG)/csrc/*.hip)
OBJ := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRC))
LIB := $(PKG)/libsv_ge2e.so
# only sv_persist.hip reads SV_FAULT_INJECTION; the other objects are shared
FAULT_OBJ := $(patsubst build/sv_persist.o,build/faultinj/sv_persist.o,$(OBJ))
FAULT_LIB := $(PKG)/libsv_ge2e_faultinj.so

all: $(LIB) $(FAULT_LIB)

# the wide-tile persistent backward keeps its MFMA accumulators in VGPRs (all AGPRs hold weights)
build/sv_persist3.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1
build/sv_persist_f32.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1

build/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/sv_ge2e.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -c $< -o $@

build/faultinj/sv_persist.o: $(PKG)/csrc/sv_persist.hip $(wildcard $(PKG)/csrc/*.h) include/sv_ge2e.h
	@mkdir -p build/faultinj
	$(HIPCC) $(CXXFLAGS) -DSV_FAULT_INJECTION -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

$(FAULT_LIB): $(FAULT_OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(FAULT_OBJ)

# A/B builds (never loaded by tests or the bench; scripts/ab/ is not sent to the GPU box unless a
# call un-ignores it): `make ab NAME=x FLAGS="-D..."` compiles every source with FLAGS into
# scripts/ab/libsv_ge2e_x.so.  The sources keep only the phase-stamp builds as flags
# (-DSV_PF32_STAMP [-DSV_PF32_WAVE_STAMP], -DSV_WB_STAMP, -DSV_WAVE3_STAMP: scripts/f32_step_ab.py
# --stamps, scripts/wave_stamps.py); a candidate kernel change is an A/B build of a patched tree
# against `make ab NAME=base FLAGS=`, timed by scripts/gpu_ab.sh.  Variants measured slower are
# deleted from the sources (DESIGN §4 keeps the record).
NAME ?= ab
FLAGS ?=
AB_OBJ := $(patsubst build/%.o,build/ab_$(NAME)/%.o,$(OBJ))
AB_LIB := scripts/ab/libsv_ge2e_$(NAME).so
build/ab_$(NAME)/sv_persist3.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1
build/ab_$(NAME)/sv_persist_f32.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1
build/ab_$(NAME)/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/sv_ge2e.h
	@mkdir -p build/ab_$(NAME)
	$(HIPCC) $(CXXFLAGS) $(EXTRA) $(FLAGS) -c $< -o $@
$(AB_LIB): $(AB_OBJ)
	@mkdir -p scripts/ab
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(AB_OBJ)
ab: $(AB_LIB)

clean:
	rm -rf build $(LIB) $(FAULT_LIB)

.PHONY: all clean ab
