# Builds the gfx950 C-ABI library (product) and the CPU oracle (test infrastructure).
#   make            -> libvfilter_hip.so + libvfdist.so + oracle
#   make tools      -> tools/tune_invert (kernel variant sweep, run on the GPU box)
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
PKG       := distributed-video-filter_amd
CSRC      := $(PKG)/csrc
LIB       := $(PKG)/vfilter/libvfilter_hip.so
DLIB      := $(PKG)/vfilter/libvfdist.so
CXX       ?= g++
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden -Wall -Iinclude
LDFLAGS   := -shared -Wl,-rpath,/opt/rocm/lib -Wl,--no-undefined

.PHONY: all lib vfdist oracle tools clean exp
all: lib oracle

lib: $(LIB) $(DLIB)

vfdist: $(DLIB)

# the distributor's native control plane: host C++ only (no HIP), so plain g++
$(DLIB): $(CSRC)/vf_dist.cc $(CSRC)/vf_json.h include/vfdist.h
	$(CXX) -O2 -g -std=c++17 -fPIC -shared -pthread -Wall -Wextra -Iinclude -fvisibility=hidden -Wl,--no-undefined $< -o $@ -lrt

SRCS := $(CSRC)/vf_kernels.hip $(CSRC)/vf_engine.hip $(CSRC)/vf_api.hip $(CSRC)/vf_jpeg_kernels.hip $(CSRC)/vf_jpeg_host.hip
HDRS := $(CSRC)/vf_internal.h $(CSRC)/vf_stream.h $(CSRC)/vf_host_mem.h $(CSRC)/vf_jpeg.h $(CSRC)/vf_jpeg_types.h $(CSRC)/vf_jpeg_parse.h $(CSRC)/vf_jpeg_codec.h include/vfilter.h

$(LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) $(LDFLAGS) -pthread $(SRCS) -o $@

oracle:
	$(MAKE) -C oracle

tools: tools/tune_invert tools/pcie_probe tools/vfd_load

tools/pcie_probe: tools/pcie_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 $< -o $@

# the native control plane driven from C++ alone (load generator, --chaos; host only)
tools/vfd_load: tools/vfd_load.cc $(DLIB) include/vfdist.h
	$(CXX) -O2 -std=c++17 -Iinclude tools/vfd_load.cc -o $@ -L$(dir $(DLIB)) -lvfdist -Wl,-rpath,$(abspath $(dir $(DLIB))) -pthread

tools/tune_invert: tools/tune_invert.hip $(CSRC)/vf_kernels.hip $(CSRC)/vf_internal.h $(CSRC)/vf_stream.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Iinclude -I$(CSRC) tools/tune_invert.hip $(CSRC)/vf_kernels.hip -o $@

clean:
	rm -f $(LIB) $(DLIB) tools/tune_invert tools/pcie_probe tools/vfd_load
	$(MAKE) -C oracle clean

# Experiment libraries (timing A/Bs against the product library; never loaded by the product):
#   make exp EXP=NAME DEFS="-DVF_EXP_...=1"  ->  tools/exp/libvf_NAME.so
exp:
	@mkdir -p tools/exp
	$(HIPCC) $(HIPFLAGS) $(DEFS) $(LDFLAGS) -pthread $(SRCS) -o tools/exp/libvf_$(EXP).so
