# Build of the MI355X batch key-hashing engine and of the parity checker.
#
#   make            -> pdht_amd/lib/libpdht_hip.so   (product: HIP kernels +
#                      C-ABI + scalar city.h API + pdht_hash shim)
#                      pdht_amd/lib/libpdht_hip_mpi.so (the same engine with
#                      the libmpipdht flavour of pdht_hash, libmpipdht/hash.c)
#                      pdht_amd/lib/libpdht_hip_tuning.so (tools/ and A/B
#                      tests: alternative kernels, -DPDHT_HIP_TUNING)
#                      oracle/liboracle.so, oracle/_ref/*.so (test checker)
#   make product    -> only the product libraries
#
# gfx950 only; plain hipcc, no CUDA/HIP dual paths.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
ARCH    ?= gfx950
LIBDIR  := pdht_amd/lib
LIB     := $(LIBDIR)/libpdht_hip.so
LIB_MPI := $(LIBDIR)/libpdht_hip_mpi.so
LIB_TUN := $(LIBDIR)/libpdht_hip_tuning.so
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden \
           -Wall -Wno-unused-function -munsafe-fp-atomics -Iinclude
CFLAGS_SHIM = -std=c99 -O3 -fPIC -fvisibility=hidden -Wall -Wextra -Iinclude

HIP_HDR := pdht_amd/csrc/city_core.h pdht_amd/csrc/kernels.h pdht_amd/csrc/bucket.h \
           include/pdht_hip.h include/pdht_city.h
SHIM_HDR := include/pdht_hash.h include/pdht_hip.h include/pdht_city.h
OBJ     := $(LIBDIR)/pdht_hip.o $(LIBDIR)/city_host.o $(LIBDIR)/pdht_hash.o
OBJ_MPI := $(LIBDIR)/pdht_hip.o $(LIBDIR)/city_host.o $(LIBDIR)/pdht_hash_mpi.o
OBJ_TUN := $(LIBDIR)/pdht_hip_tuning.o $(LIBDIR)/city_host.o $(LIBDIR)/pdht_hash.o

.PHONY: all product oracle clean asm
all: product oracle

product: $(LIB) $(LIB_MPI) $(LIB_TUN)

$(LIBDIR)/pdht_hip.o: pdht_amd/csrc/pdht_hip.hip $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/pdht_hip_tuning.o: pdht_amd/csrc/pdht_hip.hip $(HIP_HDR) pdht_amd/csrc/pdht_hip_tuning.h
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -DPDHT_HIP_TUNING -c -o $@ $<

$(LIBDIR)/city_host.o: pdht_amd/csrc/city_host.hip $(HIP_HDR)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIBDIR)/pdht_hash.o: pdht_amd/host/pdht_hash.c $(SHIM_HDR)
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS_SHIM) -c -o $@ $<

$(LIBDIR)/pdht_hash_mpi.o: pdht_amd/host/pdht_hash.c $(SHIM_HDR)
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS_SHIM) -DPDHT_HIP_MPI_FLAVOUR -c -o $@ $<

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

$(LIB_MPI): $(OBJ_MPI)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ_MPI)

$(LIB_TUN): $(OBJ_TUN)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ_TUN)

oracle:
	$(MAKE) -s -C oracle all

# ISA listing of the kernels (for register / instruction counts)
asm:
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S -o build/pdht_hip.s pdht_amd/csrc/pdht_hip.hip

clean:
	rm -f $(LIBDIR)/*.o $(LIB) $(LIB_MPI) $(LIB_TUN)
	$(MAKE) -s -C oracle clean
