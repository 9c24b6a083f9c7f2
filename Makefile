# Build the gfx950 shared library (the C-ABI of include/gpx.h) and the oracle's C checker.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := portfoliooptgp_amd/csrc
LIB := portfoliooptgp_amd/libgpx.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result

all: $(LIB)

$(CSRC)/%.o: $(CSRC)/%.hip $(CSRC)/gpx_internal.h $(CSRC)/gpx_host.h $(CSRC)/gpx_kfun.h include/gpx.h
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(CSRC)/gpx_kernels.o $(CSRC)/gpx_api.o $(CSRC)/gpx_svgp_kernels.o $(CSRC)/gpx_svgp.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $^ -o $@

clean:
	rm -f $(CSRC)/*.o $(LIB)

.PHONY: all clean
