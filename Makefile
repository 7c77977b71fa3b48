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

all: $(LIB)

$(OBJDIR)/%.o: $(SRC)/%.hip $(SRC)/common.hpp include/dbsr_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.cpp include/dbsr_hip.h
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -c $< -o $@

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
	rm -rf $(OBJDIR) $(LIB) $(PKG)/libdbsr_hip_*.so

.PHONY: all clean exp
