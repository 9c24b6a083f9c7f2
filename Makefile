# Build the gfx950 shared library (the C-ABI of include/gpx.h) and the oracle's C checker.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := portfoliooptgp_amd/csrc
LIB := portfoliooptgp_amd/libgpx.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result

CSMOKE := tests/c/gpx_c_smoke
# the L-BFGS-B driver loop in C++ (CPython extension calling scipy's setulb; lbfgsb.BatchStepper)
PYINC := $(shell python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
PYEXT := $(shell python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
LOOPMOD := portfoliooptgp_amd/_gpx_lbfgsb$(PYEXT)

all: $(LIB) $(CSMOKE) $(LOOPMOD)

$(LOOPMOD): $(CSRC)/gpx_lbfgsb_host.cpp
	g++ -O2 -std=c++17 -fPIC -shared -Wall -Wextra -Wno-missing-field-initializers -Wno-cast-function-type \
	  -I$(PYINC) $< -o $@

$(CSRC)/%.o: $(CSRC)/%.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_host.h $(CSRC)/gpx_kfun.h $(CSRC)/gpx_leaf.h $(CSRC)/gpx_b16core.h include/gpx.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# host helpers of the L-BFGS-B driver: plain gcc, libm calls as Python's math module makes them
$(CSRC)/gpx_host_math.o: $(CSRC)/gpx_host_math.c include/gpx.h
	gcc -O2 -fno-builtin -fno-fast-math -fPIC -std=c11 -Wall -c $< -o $@

$(LIB): $(CSRC)/gpx_kernels.o $(CSRC)/gpx_api.o $(CSRC)/gpx_band.o $(CSRC)/gpx_band16.o $(CSRC)/gpx_bcr.o $(CSRC)/gpx_svgp_kernels.o $(CSRC)/gpx_svgp.o $(CSRC)/gpx_host_math.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,-soname,libgpx.so $^ -o $@

# plain-C consumer of the C ABI (gcc, HIP runtime API only), run by tests/test_c_abi_gpu.py
$(CSMOKE): tests/c/gpx_c_smoke.c include/gpx.h $(LIB)
	gcc -O2 -std=c11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude $< $(LIB) \
	  -L/opt/rocm/lib -lamdhip64 -lm -Wl,-rpath,'$$ORIGIN/../../portfoliooptgp_amd' \
	  -Wl,-rpath,/opt/rocm/lib -o $@

# diagnostic variant: the fused band sweeps record per-phase shader-clock cycles
# (tools/band_phases.py loads it through GPX_LIB); never the product library
PHASES_LIB := portfoliooptgp_amd/libgpx_phases.so
$(CSRC)/gpx_band_phases.o: $(CSRC)/gpx_band.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_leaf.h $(CSRC)/gpx_kfun.h
	$(HIPCC) $(HIPFLAGS) -DGPX_BAND_PHASES -c $< -o $@
$(CSRC)/gpx_band16_phases.o: $(CSRC)/gpx_band16.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_leaf.h $(CSRC)/gpx_kfun.h
	$(HIPCC) $(HIPFLAGS) -DGPX_BAND_PHASES -c $< -o $@
$(CSRC)/gpx_bcr_phases.o: $(CSRC)/gpx_bcr.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_b16core.h $(CSRC)/gpx_kfun.h
	$(HIPCC) $(HIPFLAGS) -DGPX_BCR_PHASES -c $< -o $@
$(PHASES_LIB): $(CSRC)/gpx_kernels.o $(CSRC)/gpx_api.o $(CSRC)/gpx_band_phases.o $(CSRC)/gpx_band16_phases.o $(CSRC)/gpx_bcr_phases.o $(CSRC)/gpx_svgp_kernels.o $(CSRC)/gpx_svgp.o $(CSRC)/gpx_host_math.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -Wl,-soname,libgpx_phases.so $^ -o $@
phases: $(PHASES_LIB)

clean:
	rm -f $(CSRC)/*.o $(LIB) $(PHASES_LIB) $(CSMOKE) $(HARNESS)
	rm -rf build/asan

# host-logic harness (tests/test_host_harness.py): the library's sources compiled with
# AddressSanitizer + UndefinedBehaviorSanitizer on the HOST code only (-Xarch_host; the gfx950
# device code is built as usual and never launched: the harness calls pure host functions)
HARNESS := tests/c/host_harness
HSRC := $(wildcard $(CSRC)/*.hip)
HOBJ := $(patsubst $(CSRC)/%.hip,build/asan/%.o,$(HSRC))
HSAN := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -Xarch_host -fno-omit-frame-pointer -g -O1
build/asan/%.o: $(CSRC)/%.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_host.h $(CSRC)/gpx_kfun.h $(CSRC)/gpx_leaf.h $(CSRC)/gpx_b16core.h include/gpx.h
	@mkdir -p build/asan
	$(HIPCC) --offload-arch=$(ARCH) -std=c++17 -fPIC $(HSAN) -c $< -o $@
build/asan/gpx_host_math.o: $(CSRC)/gpx_host_math.c include/gpx.h
	@mkdir -p build/asan
	gcc -O1 -g -fno-builtin -fno-fast-math -fPIC -std=c11 -fsanitize=address,undefined -c $< -o $@
build/asan/host_harness.o: tests/c/host_harness.cpp $(CSRC)/gpx_host.h $(CSRC)/gpx_internal.h include/gpx.h
	@mkdir -p build/asan
	$(HIPCC) --offload-arch=$(ARCH) -x hip -std=c++17 $(HSAN) -Iinclude -c $< -o $@
$(HARNESS): build/asan/host_harness.o $(HOBJ) build/asan/gpx_host_math.o
	$(HIPCC) --offload-arch=$(ARCH) $(HSAN) $^ -o $@
host-harness: $(HARNESS)

.PHONY: all clean phases host-harness
