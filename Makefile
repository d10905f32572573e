# libdd.so: the MI355X (gfx950) kernels behind include/dd_capi.h
# One object per .hip (compiled in parallel with make -j), linked into one shared library.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard data_diet_distributed_amd/csrc/*.hip)
HDR := $(wildcard data_diet_distributed_amd/csrc/*.h) include/dd_capi.h
OBJDIR := build/obj
OBJ := $(patsubst data_diet_distributed_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRC))
LIB := data_diet_distributed_amd/libdd.so
HIPFLAGS := -O3 --offload-arch=$(ARCH) -std=c++17 -fPIC -Wall

all: $(LIB)

$(OBJDIR)/%.o: data_diet_distributed_amd/csrc/%.hip $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

clean:
	rm -f $(LIB) $(OBJ)

.PHONY: all clean
