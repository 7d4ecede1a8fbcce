# Top-level build: the gfx950 product library and the CPU checker (oracle, test infrastructure).
#   make            -> pyorbslam_amd/_lib/liborbfe.so + oracle/build/liborboracle.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -Wall \
            -munsafe-fp-atomics -Wno-unused-result
SRC := pyorbslam_amd/csrc/orbfe_kernels.hip pyorbslam_amd/csrc/orbfe_host.hip pyorbslam_amd/csrc/orbfe_vocab.hip
HDR := pyorbslam_amd/csrc/orbfe_common.h pyorbslam_amd/csrc/orbfe_kernels.h pyorbslam_amd/csrc/orbfe_host_util.h include/orbfe.h \
       pyorbslam_amd/csrc/brief_pattern.inc
LIB := pyorbslam_amd/_lib/liborbfe.so
OBJ := $(patsubst pyorbslam_amd/csrc/%.hip,pyorbslam_amd/_lib/%.o,$(SRC))

all: $(LIB) oracle

pyorbslam_amd/_lib/%.o: pyorbslam_amd/csrc/%.hip $(HDR)
	@mkdir -p pyorbslam_amd/_lib
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf pyorbslam_amd/_lib
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
