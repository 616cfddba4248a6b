# MI355X-native SpMV suite.  Same targets as the reference Makefile
# (reference Makefile:13: coo csr ell sigma_c cmrs -> ./bin/<fmt>), plus
# the libraries, the test oracle and test entry points.
#
#   make            libraries + the five drivers
#   make lib        libspmv_hip.so (gfx950 kernels, C-ABI) + libspmv_host.so
#   make oracle     oracle/liboracle.so (test infrastructure only)
#   make probes     libspmv_probe.so (measurement helpers: stream ceiling,
#                   flush, trace tags; never linked into the product)
#   make test-cpu   pytest -m "not gpu"
#   make test-gpu   pytest -m gpu (needs an MI355X)
#   DEBUG=yes       adds -g (reference Makefile:20-22)

PKG      := opencl-spmv-algorithms_amd
LIBDIR   := $(PKG)/lib
BINDIR   := bin
HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
ARCH     ?= gfx950
ROCM     ?= /opt/rocm

CFLAGS   := -O3 -std=c11 -Wall -Wextra -Werror -Wshadow -fPIC -fopenmp -Iinclude
HIPFLAGS := -O3 -std=c++17 -Wall -Wextra -fPIC --offload-arch=$(ARCH) -Iinclude
ifeq ($(DEBUG), yes)
CFLAGS   += -g
HIPFLAGS += -g
endif

HIP_SRC  := $(wildcard $(PKG)/csrc/*.hip)
HIP_HDR  := $(wildcard $(PKG)/csrc/*.h) include/spmv.h include/spmv_rc.h
HOST_SRC := $(wildcard $(PKG)/host/*.c)
TARGETS  := coo csr ell sigma_c cmrs

LIB_HIP  := $(LIBDIR)/libspmv_hip.so
LIB_HOST := $(LIBDIR)/libspmv_host.so
ORACLE   := oracle/liboracle.so

.PHONY: all default lib oracle probes test-cpu test-gpu clean $(TARGETS)

default: all
all: lib $(TARGETS) probes

lib: $(LIB_HIP) $(LIB_HOST)

# one object per .hip (parallel with make -j), linked into one library
HIP_OBJ  := $(patsubst $(PKG)/csrc/%.hip,build/hip/%.o,$(HIP_SRC))

build/hip/%.o: $(PKG)/csrc/%.hip $(HIP_HDR)
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB_HIP): $(HIP_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(HIP_OBJ) -o $@

$(LIB_HOST): $(HOST_SRC) include/spmv_host.h include/spmv_rc.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -shared $(HOST_SRC) -o $@ -lm

$(TARGETS): %: $(BINDIR)/%

$(BINDIR)/%: $(PKG)/drivers/%.c $(PKG)/drivers/driver.c $(PKG)/drivers/driver.h $(LIB_HIP) $(LIB_HOST)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -I$(PKG)/drivers $< $(PKG)/drivers/driver.c -o $@ \
	  -L$(LIBDIR) -lspmv_hip -lspmv_host -Wl,-rpath,'$$ORIGIN/../$(LIBDIR)' \
	  -Wl,-rpath,$(ROCM)/lib -lm

oracle: $(ORACLE)

LIB_PROBE := $(LIBDIR)/libspmv_probe.so
probes: $(LIB_PROBE)

$(LIB_PROBE): tools/probe.hip
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $< -o $@

$(ORACLE): oracle/oracle.c
	$(CC) -O2 -std=c11 -Wall -Wextra -fPIC -fopenmp -shared $< -o $@ -lm

test-cpu: all oracle
	python -m pytest tests/ -x -q -m "not gpu"

test-gpu: all oracle
	python -m pytest tests/ -x -q -m gpu

clean:
	$(RM) -r $(BINDIR) $(LIBDIR) $(ORACLE) build
