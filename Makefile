# Build of the MI355X (gfx950) admission engine. `python -c "import __graft_entry__ as g; g.build()"`
# runs this; hipcc cross-compiles for gfx950 without a GPU.
#   policy-server_amd/libkwgpu.so    product: HIP kernels + host engine + C ABI (include/kwgpu.h)
#   policy-server_amd/libkwsynth.so  bench/test workload generator
#   policy-server_amd/kwhost         HTTP front (/validate, /audit, /validate_raw) over libkwgpu.so
#   policy-server_amd/kwload         closed-loop HTTP load generator for kwhost (serving measurement)
#   oracle/build/libkworacle.so      CPU restatement (test infrastructure only)
HIPCC ?= /opt/rocm/bin/hipcc
CXX ?= g++
CC ?= gcc
ARCH ?= gfx950
PKG := policy-server_amd
SRC := $(PKG)/csrc
OBJ := $(PKG)/build
HIPDEF := -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Wextra $(HIPDEF)
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -munsafe-fp-atomics $(HIPEXTRA)

HOST_SRCS := json yaml automaton expr env flatten service slotplan metrics capi
HOST_OBJS := $(addprefix $(OBJ)/,$(addsuffix .o,$(HOST_SRCS)))
HEADERS := $(wildcard $(SRC)/*.hpp) include/kwgpu.h

all: $(PKG)/libkwgpu.so $(PKG)/libkwsynth.so $(PKG)/kwhost $(PKG)/kwload oracle/build/libkworacle.so scripts/lds_calib scripts/lds_occ scripts/fmt_bench

# kwhost's host stages (flatten, response JSON) timed without a GPU
scripts/fmt_bench: scripts/fmt_bench.cpp include/kwgpu.h $(PKG)/libkwgpu.so $(PKG)/libkwsynth.so
	$(CXX) -O2 -std=c++17 $< -o $@ -L$(PKG) -lkwgpu -lkwsynth -Wl,-rpath,'$$ORIGIN/../$(PKG)'

# LDS counter calibration micro-kernels (scripts/lds_calib.sh runs them under rocprofv3 --pmc)
scripts/lds_calib: scripts/lds_calib.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -o $@ $<

# LDS residency probe: workgroups a CU holds per dynamic LDS size (profiles/r05_lds_residency.txt)
scripts/lds_occ: scripts/lds_occ.hip
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -o $@ $<

$(OBJ)/%.o: $(SRC)/%.cpp $(HEADERS)
	@mkdir -p $(OBJ)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(OBJ)/kernels.o: $(SRC)/kernels.hip $(HEADERS)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(PKG)/libkwgpu.so: $(HOST_OBJS) $(OBJ)/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(PKG)/kwhost: $(SRC)/kwhost.cpp include/kwgpu.h $(PKG)/libkwgpu.so
	$(CXX) -O2 -std=c++17 -Wall -Wextra -o $@ $< -L$(PKG) -lkwgpu -Wl,-rpath,'$$ORIGIN' -lpthread

$(PKG)/kwload: $(SRC)/kwload.cpp $(PKG)/libkwsynth.so
	$(CXX) -O2 -std=c++17 -Wall -Wextra -o $@ $< -L$(PKG) -lkwsynth -Wl,-rpath,'$$ORIGIN' -lpthread

$(PKG)/libkwsynth.so: $(SRC)/synth.cpp include/kwgpu.h
	$(CXX) -O3 -std=c++17 -fPIC -shared -Wall -o $@ $<

oracle/build/libkworacle.so: oracle/kworacle.c oracle/kwregex.c oracle/kworacle.h oracle/unicode_data.h include/kwgpu.h
	@mkdir -p oracle/build
	$(CC) -O2 -std=c11 -fPIC -shared -Wall -Wextra -o $@ oracle/kworacle.c oracle/kwregex.c -lpthread

# A/B variant of the library with extra kernel flags: make variant NAME=x VFLAGS="-DKW_PREFETCH=0"
# -> policy-server_amd/variants/x.so (KWGPU_LIB selects it; scripts/ab.sh benches every variant);
# KSRC=<file in csrc/> builds another kernels source (e.g. the previous commit's)
variant: $(HOST_OBJS)
	@mkdir -p $(PKG)/variants/obj-$(NAME)
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $(or $(KSRC),$(SRC)/kernels.hip) -o $(PKG)/variants/obj-$(NAME)/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(PKG)/variants/$(NAME).so $(HOST_OBJS) $(PKG)/variants/obj-$(NAME)/kernels.o

# A/B variant built entirely (host engine + kernels) from another source directory next to csrc/,
# e.g. a snapshot of an earlier commit: make variant-full NAME=x VSRC=policy-server_amd/csrc_x
variant-full:
	@mkdir -p $(PKG)/variants/obj-$(NAME)
	for f in $(HOST_SRCS); do $(CXX) $(CXXFLAGS) $(VFLAGS) -c $(VSRC)/$$f.cpp -o $(PKG)/variants/obj-$(NAME)/$$f.o || exit 1; done
	$(HIPCC) $(HIPFLAGS) $(VFLAGS) -c $(VSRC)/kernels.hip -o $(PKG)/variants/obj-$(NAME)/kernels.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(PKG)/variants/$(NAME).so $(addprefix $(PKG)/variants/obj-$(NAME)/,$(addsuffix .o,$(HOST_SRCS))) $(PKG)/variants/obj-$(NAME)/kernels.o

# kernel resource usage (VGPR/SGPR/LDS/occupancy) report
resources: $(SRC)/kernels.hip
	$(HIPCC) $(HIPFLAGS) -Rpass-analysis=kernel-resource-usage -c $< -o /dev/null

clean:
	rm -rf $(OBJ) $(PKG)/*.so $(PKG)/kwhost $(PKG)/kwload oracle/build

.PHONY: all clean resources variant
