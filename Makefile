# libdd.so: the MI355X (gfx950) kernels behind include/dd_capi.h
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
SRC := $(wildcard data_diet_distributed_amd/csrc/*.hip)
HDR := $(wildcard data_diet_distributed_amd/csrc/*.h) include/dd_capi.h
LIB := data_diet_distributed_amd/libdd.so
HIPFLAGS := -O3 --offload-arch=$(ARCH) -std=c++17 -fPIC -shared -Wall

all: $(LIB)

$(LIB): $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC)

clean:
	rm -f $(LIB)

.PHONY: all clean
