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
HIP_HDR  := $(wildcard $(PKG)/csrc/*.h) include/spmv.h include/spmv_ext.h include/spmv_host.h include/spmv_rc.h
HOST_SRC := $(wildcard $(PKG)/host/*.c)
TARGETS  := coo csr ell sigma_c cmrs

LIB_HIP  := $(LIBDIR)/libspmv_hip.so
LIB_HOST := $(LIBDIR)/libspmv_host.so
ORACLE   := oracle/liboracle.so

.PHONY: all default lib oracle probes lab test-san test-cpu test-gpu clean $(TARGETS)

default: all
all: lib $(TARGETS) probes

lib: $(LIB_HIP) $(LIB_HOST)

# one object per .hip (parallel with make -j), linked into one library
HIP_OBJ  := $(patsubst $(PKG)/csrc/%.hip,build/hip/%.o,$(HIP_SRC))

build/hip/%.o: $(PKG)/csrc/%.hip $(HIP_HDR)
	@mkdir -p build/hip
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the plans (csrc/plan.hip) call the host rules of libspmv_host.so
# (variant rules, SELL split plan, tiled-CSR big-tile plan): linked by soname
# and found next to libspmv_hip.so ($ORIGIN)
$(LIB_HIP): $(HIP_OBJ) $(LIB_HOST)
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $(HIP_OBJ) -o $@ -L$(LIBDIR) -lspmv_host -Wl,-rpath,'$$ORIGIN' -ldl

$(LIB_HOST): $(HOST_SRC) include/spmv_host.h include/spmv_rc.h
	@mkdir -p $(LIBDIR)
	$(CC) $(CFLAGS) -shared $(HOST_SRC) -o $@ -Wl,-soname,libspmv_host.so -lm

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

# diagnostic kernel copies with per-wave timestamps (tools/*_lab.*)
lab: $(LIBDIR)/libspmv_lab.so

$(LIBDIR)/libspmv_lab.so: tools/sell_lab.hip
	@mkdir -p $(LIBDIR)
	$(HIPCC) $(HIPFLAGS) -shared $< -o $@

$(ORACLE): oracle/oracle.c
	$(CC) -O2 -std=c11 -Wall -Wextra -fPIC -fopenmp -shared $< -o $@ -lm

test-cpu: all oracle
	python -m pytest tests/ -x -q -m "not gpu"
ifeq ($(SAN), 1)
	$(MAKE) test-san
endif

# ---- host sanitizers: the host library, the oracle and the
# drivers' host code built with ASan + UBSan, run over the fixtures, malformed
# files and the generators (tests/san/host_harness.c), under the host and
# oracle pytest suites, and as the five programs (no GPU here: they must stop
# with the reference's device error, 1, after parsing and building)
SANFLAGS := -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=all
SANENV   := ASAN_OPTIONS=detect_leaks=0:exitcode=99 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:exitcode=99
LIBASAN  := $(shell $(CC) -print-file-name=libasan.so)
SAN_BIN  := $(addprefix build/san/bin/,$(TARGETS))

build/san/host_harness: tests/san/host_harness.c $(HOST_SRC) include/spmv_host.h include/spmv_rc.h
	@mkdir -p build/san
	$(CC) -std=c11 -Wall -Wextra -Werror -fopenmp -Iinclude $(SANFLAGS) $< $(HOST_SRC) -o $@ -lm

build/san/libspmv_host.so: $(HOST_SRC) include/spmv_host.h include/spmv_rc.h
	@mkdir -p build/san
	$(CC) -std=c11 -Wall -Wextra -Werror -fPIC -fopenmp -Iinclude $(SANFLAGS) -shared $(HOST_SRC) -o $@ -lm

build/san/liboracle.so: oracle/oracle.c
	@mkdir -p build/san
	$(CC) -std=c11 -Wall -Wextra -fPIC -fopenmp $(SANFLAGS) -shared $< -o $@ -lm

build/san/bin/%: $(PKG)/drivers/%.c $(PKG)/drivers/driver.c $(PKG)/drivers/driver.h $(HOST_SRC) $(LIB_HIP)
	@mkdir -p build/san/bin
	$(CC) -std=c11 -Wall -Wextra -Werror -Wshadow -fopenmp -Iinclude -I$(PKG)/drivers $(SANFLAGS) $< \
	  $(PKG)/drivers/driver.c $(HOST_SRC) -o $@ -L$(LIBDIR) -lspmv_hip -Wl,-rpath,$(abspath $(LIBDIR)) \
	  -Wl,-rpath,$(ROCM)/lib -lm

test-san: build/san/host_harness build/san/libspmv_host.so build/san/liboracle.so $(SAN_BIN)
	$(SANENV) ASAN_OPTIONS=detect_leaks=1:exitcode=99 build/san/host_harness $${TMPDIR:-/tmp} tests/golden/*.mtx
	LD_PRELOAD=$(LIBASAN) $(SANENV) SPMV_HOST_LIB=$(abspath build/san/libspmv_host.so) \
	  SPMV_ORACLE_LIB=$(abspath build/san/liboracle.so) python -m pytest tests/test_host.py tests/test_oracle.py \
	  -x -q -p no:cacheprovider
	@for f in $(TARGETS); do for m in tests/golden/empty_rows.mtx tests/golden/n67.mtx tests/golden/longest_last.mtx; do \
	  $(SANENV) build/san/bin/$$f --matrix $$m > build/san/$$f.log 2>&1; rc=$$?; \
	  if [ $$rc -ne 0 ] && [ $$rc -ne 1 ]; then echo "$$f $$m: exit $$rc"; cat build/san/$$f.log; exit 1; fi; \
	done; done; echo "sanitized drivers: clean (exit 0 on a GPU; 1 = no GPU found, before any input is read)"

test-gpu: all oracle
	python -m pytest tests/ -x -q -m gpu

clean:
	$(RM) -r $(BINDIR) $(LIBDIR) $(ORACLE) build
