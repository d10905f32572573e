# libdd.so: the MI355X (gfx950) kernels behind include/dd_capi.h
# One object per .hip (compiled in parallel with make -j), linked into one shared library.
HIPCC ?= /opt/rocm/bin/hipcc
# target-id-neutral gfx950 code object: loads whatever the device's XNACK mode.  (An
# xnack- object measured +2-3 % on the 64-channel conv and 32->16 down kernels,
# profiles/r02_v2/experiments/xnack_*, but would not load on an XNACK-on device.)
ARCHFLAGS ?= --offload-arch=gfx950
SRC := $(wildcard data_diet_distributed_amd/csrc/*.hip)
HDR := $(wildcard data_diet_distributed_amd/csrc/*.h) include/dd_capi.h Makefile
OBJDIR := build/obj
OBJ := $(patsubst data_diet_distributed_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRC))
LIB := data_diet_distributed_amd/libdd.so
HIPFLAGS := -O3 $(ARCHFLAGS) -std=c++17 -fPIC -Wall

all: $(LIB)

$(OBJDIR)/%.o: data_diet_distributed_amd/csrc/%.hip $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) $(ARCHFLAGS) -shared -fPIC -o $@ $(OBJ)

clean:
	rm -f $(LIB) $(OBJ)

.PHONY: all clean
