# Top-level build: the gfx950 product library and the CPU checker (oracle, test infrastructure).
#   make            -> pyorbslam_amd/_lib/liborbfe.so + oracle/build/liborboracle.so
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math -Wall \
            -munsafe-fp-atomics -Wno-unused-result
SRC := pyorbslam_amd/csrc/orbfe_kernels.hip pyorbslam_amd/csrc/orbfe_host.hip pyorbslam_amd/csrc/orbfe_vocab.hip
CSRC := pyorbslam_amd/csrc/orbfe_png.cpp
HDR := pyorbslam_amd/csrc/orbfe_common.h pyorbslam_amd/csrc/orbfe_kernels.h pyorbslam_amd/csrc/orbfe_host_util.h include/orbfe.h \
       pyorbslam_amd/csrc/brief_pattern.inc
LIB := pyorbslam_amd/_lib/liborbfe.so
OBJ := $(patsubst pyorbslam_amd/csrc/%.hip,pyorbslam_amd/_lib/%.o,$(SRC)) \
       $(patsubst pyorbslam_amd/csrc/%.cpp,pyorbslam_amd/_lib/%.o,$(CSRC))

# host-side CPython extension (no device code): the per-frame Python objects of the reference data model
PY := python3
PYHOST := pyorbslam_amd/_pyhost$(shell $(PY) -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC := $(shell $(PY) -c "import sysconfig, numpy; print('-I' + sysconfig.get_paths()['include'], '-I' + numpy.get_include())")

all: $(LIB) $(PYHOST) oracle

$(PYHOST): pyorbslam_amd/csrc/orbfe_pyhost.cpp
	g++ -O2 -std=c++17 -fPIC -shared -Wall $(PYINC) -o $@ $<

pyorbslam_amd/_lib/%.o: pyorbslam_amd/csrc/%.hip $(HDR)
	@mkdir -p pyorbslam_amd/_lib
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# host-only C++ (ingest): no device code
pyorbslam_amd/_lib/%.o: pyorbslam_amd/csrc/%.cpp $(HDR)
	@mkdir -p pyorbslam_amd/_lib
	$(HIPCC) -O3 -std=c++17 -fPIC -Wall -x c++ -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -c -o $@ $<

# orbfe_build_id(): the hash of every source and header and of the compiler flags (a variant build with
# extra -D switches gets its own id), regenerated whenever the library is relinked
BUILD_ID_O := pyorbslam_amd/_lib/build_id.o
$(LIB): $(OBJ)
	@printf 'const char* orbfe_build_id(void) { return "%s"; }\n' "$$( (cat $(SRC) $(CSRC) $(HDR); echo '$(HIPFLAGS)') | sha256sum | cut -c1-16)" \
	  > pyorbslam_amd/_lib/build_id.c
	gcc -O2 -fPIC -c -o $(BUILD_ID_O) pyorbslam_amd/_lib/build_id.c
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(OBJ) $(BUILD_ID_O) -lz -lpthread

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -rf pyorbslam_amd/_lib $(PYHOST)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
