# Builds the product library (HIP kernels + C ABI) for gfx950, in-tree.
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
PKG     := deep-rawburst-sr_amd
SRC     := $(PKG)/csrc
OBJDIR  := $(PKG)/build
LIB     := $(PKG)/libdbsr_hip.so
HIPSRCS := $(wildcard $(SRC)/*.hip)
CPPSRCS := $(wildcard $(SRC)/*.cpp)
OBJS    := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.o,$(HIPSRCS)) $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(CPPSRCS))
FLAGS   := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -Wall -Wno-unused-function

# torch.ops.dbsr.* operator library (TORCH_LIBRARY over the C ABI; loaded by dbsr_amd/torch_ops.py)
TORCH_DIR := $(shell python3 -c "import torch, os; print(os.path.dirname(torch.__file__))")
TORCH_LIB := $(PKG)/libdbsr_torch.so
TORCH_FLAGS := --offload-arch=$(ARCH) -O2 -std=c++17 -fPIC -D_GLIBCXX_USE_CXX11_ABI=1 -DUSE_ROCM=1 \
	-I$(TORCH_DIR)/include -I$(TORCH_DIR)/include/torch/csrc/api/include -Iinclude -Wno-unused-result \
	-Wno-deprecated-declarations

all: $(LIB) $(TORCH_LIB)

$(OBJDIR)/%.o: $(SRC)/%.hip $(SRC)/common.hpp $(SRC)/conv_core.hpp include/dbsr_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.cpp include/dbsr_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -c $< -o $@

# No SLP vectorisation for the fused weight-predictor kernel: ROCm 7.2's gfx950 code emitted a packed-fp32
# v_pk_mul_f32 that overwrote a 16-B buffer store's data registers right after the store, and the store wrote
# the new values for part of the wave; scalar fp32 ops are also the cheaper ones beside MFMAs.
$(OBJDIR)/conv_fuse.o: FLAGS += -fno-slp-vectorize

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# Experiment build: same sources with extra -D flags, loaded via DBSR_HIP_LIB for A/B profiling.
EXP_FLAGS ?=
EXP_NAME  ?= exp
EXP_LIB   := $(PKG)/libdbsr_hip_$(EXP_NAME).so
exp:
	@mkdir -p $(OBJDIR)/$(EXP_NAME)
	for f in $(HIPSRCS) $(CPPSRCS); do \
	  $(HIPCC) $(FLAGS) $(EXP_FLAGS) -c $$f -o $(OBJDIR)/$(EXP_NAME)/$$(basename $$f).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(EXP_LIB) $(OBJDIR)/$(EXP_NAME)/*.o

clean:
	rm -rf $(OBJDIR) $(LIB) $(TORCH_LIB) $(PKG)/libdbsr_hip_*.so

.PHONY: all clean exp

torchops: $(TORCH_LIB)
$(TORCH_LIB): $(SRC)/torch/torch_ops.cpp include/dbsr_hip.h $(LIB)
	$(HIPCC) $(TORCH_FLAGS) -shared -o $@ $(SRC)/torch/torch_ops.cpp -L$(TORCH_DIR)/lib -lc10 -lc10_hip -ltorch \
		-ltorch_cpu -ltorch_hip -L$(PKG) -ldbsr_hip -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,$(TORCH_DIR)/lib
.PHONY: torchops
