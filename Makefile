# Build of the MI355X batch key-hashing engine and of the parity checker.
#
#   make            -> pdht_amd/lib/libpdht_hip.so   (product: HIP kernels +
#                      C-ABI + scalar city.h API + pdht_hash shim)
#                      oracle/liboracle.so, oracle/_ref/*.so (test checker)
#   make product    -> only the product library
#
# gfx950 only; plain hipcc, no CUDA/HIP dual paths.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
LIBDIR  := pdht_amd/lib
LIB     := $(LIBDIR)/libpdht_hip.so
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden \
           -Wall -Wno-unused-function -munsafe-fp-atomics -Iinclude
CFLAGS_SHIM = -std=c99 -O3 -fPIC -fvisibility=hidden -Wall -Wextra -Iinclude

HIP_SRC := pdht_amd/csrc/pdht_hip.hip pdht_amd/csrc/city_host.hip
HIP_HDR := pdht_amd/csrc/city_core.h pdht_amd/csrc/kernels.h pdht_amd/csrc/bucket.h \
           include/pdht_hip.h include/pdht_city.h
OBJ     := $(LIBDIR)/pdht_hip.o $(LIBDIR)/city_host.o $(LIBDIR)/pdht_hash.o

.PHONY: all product oracle clean asm
all: product oracle

product: $(LIB)

$(LIBDIR)/pdht_hip.o: pdht_amd/csrc/pdht_hip.hip $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/city_host.o: pdht_amd/csrc/city_host.hip $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/pdht_hash.o: pdht_amd/host/pdht_hash.c include/pdht_hash.h include/pdht_hip.h include/pdht_city.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS_SHIM) -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

oracle:
	$(MAKE) -s -C oracle all

# ISA listing of the kernels (for register / instruction counts)
asm:
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/pdht_hip.s pdht_amd/csrc/pdht_hip.hip

clean:
	rm -f $(OBJ) $(LIB)
	$(MAKE) -s -C oracle clean
