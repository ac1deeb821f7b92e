# Build-container-only targets of harness/Makefile (never needed on the GPU
# box: gpurun-ignored together with their outputs).

# The config 4 fixture's builder (tests/make_cstr_fixture.sh): the same
# unchanged sources against a real LAPACK -- SciPy's bundled OpenBLAS, whose
# LAPACKE entry points carry a scipy_ prefix -- so the
# fixture does not depend on this repository's LAPACKE subset.
SCIPY_LIBS ?= $(shell python3 -c "import scipy, os; print(os.path.join(os.path.dirname(scipy.__file__), '..', 'scipy.libs'))" 2>/dev/null)
OPENBLAS    = $(firstword $(wildcard $(SCIPY_LIBS)/libscipy_openblas*.so))
SCIPY_RENAME := $(foreach f,dgetrf dgetri zgetrf zgetri zgeev dgesvd,-DLAPACKE_$(f)=scipy_LAPACKE_$(f))

ref-openblas: $(OUT)/openblas/cstr-run

$(OUT)/openblas/cstr-run: cstr_run.c $(addprefix $(REF)/src/,$(HECTR_SRCS)) $(ROOT)/oracle/libgpqhe_oracle.so
	@test -n "$(OPENBLAS)" || { echo "SciPy's OpenBLAS not found"; exit 1; }
	@mkdir -p $(OUT)/openblas
	ln -sf ../../libgpqhe_oracle.so $(OUT)/openblas/libgpqhe.so
	$(CC) $(CFLAGS_REF) $(SCIPY_RENAME) $(addprefix $(REF)/src/,$(HECTR_SRCS)) -fPIC -shared \
	  $(OPENBLAS) -Wl,-rpath,$(dir $(OPENBLAS)) -lm -o $(OUT)/openblas/libhectr.so
	$(CC) -O2 -std=gnu11 -Wall -Wextra -I$(REF)/src -I$(ROOT)/src -I$(ROOT)/harness/include cstr_run.c -L$(OUT)/openblas -L$(LIB) \
	  -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../harness/lib' -lhectr -lgpqhe -lpmu -lm -o $@

# Diagnostic build (CPU only, build container): the same unchanged sources and
# driver with AddressSanitizer in recover mode over the CPU oracle.  At N = 100
# ctr_hempc writes 33 rows into a 32 x 32 stack matrix (reference
# src/hempc.c:233-234 -> d2z_matrix, src/matrices.c:140); here the stray
# write lands in a redzone instead of on a live neighbour (tests/test_cstr_driver.py).
ASAN := -O0 -g -fsanitize=address -fsanitize-recover=address -fno-omit-frame-pointer
ref-asan: $(OUT)/asan/cstr-run

$(OUT)/asan/cstr-run: cstr_run.c $(addprefix $(REF)/src/,$(HECTR_SRCS)) $(ROOT)/oracle/libgpqhe_oracle.so $(LIB)/liblapacke.so $(LIB)/libpmu.so
	@mkdir -p $(OUT)/asan
	ln -sf ../../libgpqhe_oracle.so $(OUT)/asan/libgpqhe.so
	$(CC) $(ASAN) -I$(ROOT)/src -I$(ROOT)/harness/include $(addprefix $(REF)/src/,$(HECTR_SRCS)) -fPIC -shared \
	  -L$(LIB) -Wl,-rpath,'$$ORIGIN/../../../harness/lib' -llapacke -lm -o $(OUT)/asan/libhectr.so 2> /dev/null
	$(CC) $(ASAN) -std=gnu11 -I$(REF)/src -I$(ROOT)/src -I$(ROOT)/harness/include cstr_run.c -L$(OUT)/asan -L$(LIB) \
	  -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,'$$ORIGIN/../../../harness/lib' -lhectr -lgpqhe -lpmu -llapacke -lm -o $@

.PHONY: ref-openblas ref-asan
