# Builds the gfx950 HIP library behind the C ABI in include/sv_ge2e.h.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CXXFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
PKG := pytorch_speaker_verification_amd
SRC := $(wildcard $(PKG)/csrc/*.hip)
OBJ := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRC))
LIB := $(PKG)/libsv_ge2e.so

all: $(LIB)

# the wide-tile persistent backward keeps its MFMA accumulators in VGPRs (all AGPRs hold weights)
build/sv_persist3.o: EXTRA := -mllvm -amdgpu-mfma-vgpr-form=1

build/%.o: $(PKG)/csrc/%.hip $(wildcard $(PKG)/csrc/*.h) include/sv_ge2e.h
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) $(EXTRA) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
