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

clean:
	rm -rf $(OBJDIR) $(LIB)

.PHONY: all clean
