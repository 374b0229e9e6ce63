# Build of the MI355X batch key-hashing engine and of the parity checker.
#
#   make            -> pdht_amd/lib/libpdht_hip.so   (product: HIP kernels +
#                      C-ABI + scalar city.h API + pdht_hash shim)
#                      pdht_amd/lib/libpdht_hip_mpi.so (the same engine with
#                      the libmpipdht flavour of pdht_hash, libmpipdht/hash.c)
#                      pdht_amd/lib/libpdht_hip_tuning.so (tools/ and A/B
#                      tests: the same sources with the A/B hook headers of
#                      pdht_amd/csrc/tuning/ instead of pdht_amd/csrc/product/)
#                      oracle/liboracle.so, oracle/_ref/*.so (test checker)
#   make product    -> only the product libraries
#
# gfx950 only; plain hipcc, no CUDA/HIP dual paths.

HIPCC   ?= /opt/rocm/bin/hipcc
CC      ?= gcc
# gfx950 only: the kernels size their LDS for its 160 KiB per CU (e.g.
# k_bucket_base stages 64 KiB of totals), which other targets do not have
ARCH    := gfx950
LIBDIR  := pdht_amd/lib
LIB     := $(LIBDIR)/libpdht_hip.so
LIB_MPI := $(LIBDIR)/libpdht_hip_mpi.so
LIB_TUN := $(LIBDIR)/libpdht_hip_tuning.so
HIPFLAGS = --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden \
           -Wall -Wno-unused-function -munsafe-fp-atomics -Iinclude
# "pdht_hooks*.h": the product's (every A/B hook a no-op) or the tuning build's
HOOKS_PRODUCT := -Ipdht_amd/csrc/product
HOOKS_TUNING  := -Ipdht_amd/csrc/tuning
CFLAGS_SHIM = -std=c99 -O3 -fPIC -fvisibility=hidden -Wall -Wextra -Iinclude

HIP_HDR := pdht_amd/csrc/city_core.h pdht_amd/csrc/kernels.h pdht_amd/csrc/runtime.h \
           pdht_amd/csrc/bucket.h pdht_amd/csrc/launch.h include/pdht_hip.h include/pdht_city.h
HDR_PRODUCT := $(wildcard pdht_amd/csrc/product/*.h)
HDR_TUNING := $(wildcard pdht_amd/csrc/tuning/*.h) pdht_amd/csrc/pdht_hip_tuning.h
SHIM_HDR := include/pdht_hash.h include/pdht_hip.h include/pdht_city.h
# the C-ABI in translation units that build in parallel (make -j)
HIP_UNITS := pdht_hip pdht_fixed64 pdht_fixed128 pdht_var pdht_host pdht_bucket
OBJ_ENG := $(HIP_UNITS:%=$(LIBDIR)/%.o) $(LIBDIR)/city_host.o
OBJ_TUN_ENG := $(HIP_UNITS:%=$(LIBDIR)/%.tun.o) $(LIBDIR)/city_host.o $(LIBDIR)/pdht_tuning.tun.o
OBJ     := $(OBJ_ENG) $(LIBDIR)/pdht_hash.o
OBJ_MPI := $(OBJ_ENG) $(LIBDIR)/pdht_hash_mpi.o
OBJ_TUN := $(OBJ_TUN_ENG) $(LIBDIR)/pdht_hash.o

# Compile-time experiments for tools/abbench.py (`--variants x0` = variant 0
# of this build): the tuning build plus EXP flags, e.g.
#   make exp EXP=-DPDHT_COUNT_NT=false [EXP_TAG=cnt -> libpdht_hip_exp_cnt.so, `--variants x0:cnt`]
EXP ?=
EXP_TAG ?=
LIB_EXP := $(LIBDIR)/libpdht_hip_exp$(if $(EXP_TAG),_$(EXP_TAG)).so
OBJ_EXP := $(HIP_UNITS:%=$(LIBDIR)/%.exp.o) $(LIBDIR)/city_host.o $(LIBDIR)/pdht_tuning.tun.o $(LIBDIR)/pdht_hash.o

.PHONY: all product oracle clean asm exp
all: product oracle

product: $(LIB) $(LIB_MPI) $(LIB_TUN)

# unit-specific headers
$(LIBDIR)/pdht_bucket.o $(LIBDIR)/pdht_bucket.tun.o: pdht_amd/csrc/bucket.h
$(foreach u,pdht_fixed64 pdht_fixed128 pdht_var pdht_host,$(LIBDIR)/$(u).o $(LIBDIR)/$(u).tun.o): pdht_amd/csrc/launch.h

# (product objects never see the tuning headers, and the reverse)
$(LIBDIR)/%.o: pdht_amd/csrc/%.hip $(HIP_HDR) $(HDR_PRODUCT)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(HOOKS_PRODUCT) -c -o $@ $<

$(LIBDIR)/%.tun.o: pdht_amd/csrc/%.hip $(HIP_HDR) $(HDR_TUNING)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(HOOKS_TUNING) -c -o $@ $<

$(LIBDIR)/pdht_tuning.tun.o: pdht_amd/csrc/tuning/pdht_tuning.hip $(HIP_HDR) $(HDR_TUNING)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(HOOKS_TUNING) -c -o $@ $<

$(LIBDIR)/%.exp.o: pdht_amd/csrc/%.hip $(HIP_HDR) $(HDR_TUNING) FORCE
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) $(HOOKS_TUNING) $(EXP) -c -o $@ $<

exp: $(OBJ_EXP)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIB_EXP) $(OBJ_EXP)

FORCE:

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
	for u in $(HIP_UNITS); do $(HIPCC) $(HIPFLAGS) $(HOOKS_PRODUCT) --cuda-device-only -S -o build/$$u.s pdht_amd/csrc/$$u.hip || exit 1; done

clean:
	rm -f $(LIBDIR)/*.o $(LIB) $(LIB_MPI) $(LIB_TUN) $(LIBDIR)/libpdht_hip_exp*.so
	$(MAKE) -s -C oracle clean
