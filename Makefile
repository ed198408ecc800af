# libgeoflink_hip.so -- MI355X (gfx950) window-evaluation hot path, plus the test oracle.
# -ffp-contract=off on host AND device: Java never fuses a*b+c, and the exact prefilters
# (smax, cell thresholds) must see the same rounding on both sides.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -ffp-contract=off -fno-fast-math \
            -Wall -Wno-unused-function -Wno-unused-result -Wno-unused-value
SRC      := spatialflink_amd/csrc
OBJDIR   := build/obj
LIB      := spatialflink_amd/libgeoflink_hip.so
SOURCES  := $(SRC)/api.cpp $(SRC)/comm.cpp $(SRC)/sliding.cpp $(SRC)/csv.cpp $(SRC)/objid.cpp $(SRC)/k_points.hip $(SRC)/k_knn.hip \
            $(SRC)/k_range.hip $(SRC)/k_join.hip $(SRC)/k_csv.hip $(SRC)/k_objid.hip
OBJECTS  := $(patsubst $(SRC)/%,$(OBJDIR)/%.o,$(SOURCES))
HEADERS  := include/geoflink_hip.h $(SRC)/gf_buildtag.hpp $(SRC)/gf_internal.hpp $(SRC)/gf_text.hpp $(SRC)/gf_geojson.hpp $(SRC)/gf_numerics.hpp $(SRC)/gf_decimal.hpp $(SRC)/gf_pow5.hpp $(SRC)/gf_geom.hpp

all: $(LIB) oracle shim

# the plain-C core of the JNI shim (integration/jni/geoflink_shim.c) as a library the tests drive
# through ctypes exactly as geoflink_jni.c's natives call it (no JDK in the image)
SHIM     := integration/jni/libgeoflink_shim.so
$(SHIM): integration/jni/geoflink_shim.c integration/jni/geoflink_shim.h include/geoflink_hip.h $(LIB)
	gcc -O2 -std=c11 -Wall -Wextra -Werror -fPIC -shared -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
	    $< -o $@ -Lspatialflink_amd -lgeoflink_hip -L/opt/rocm/lib -lamdhip64 \
	    -Wl,-rpath,'$$ORIGIN/../../spatialflink_amd' -Wl,-rpath,/opt/rocm/lib
shim: $(SHIM)

# The product rule takes no extra defines: experiments build only into
# explibs/ through tools/build_exp.sh.  The flags stamp is rewritten at parse time whenever the
# compile line differs from the last build's, so a changed HIPFLAGS (e.g. `make HIPFLAGS=...-DX`)
# rebuilds every object, and the next plain `make` rebuilds them again as the product.
FLAGS_STAMP := $(OBJDIR)/.hipflags
$(shell mkdir -p $(OBJDIR); printf '%s\n' '$(HIPCC) $(HIPFLAGS)' | cmp -s - $(FLAGS_STAMP) || \
        printf '%s\n' '$(HIPCC) $(HIPFLAGS)' > $(FLAGS_STAMP))
$(OBJDIR)/%.o: $(SRC)/% $(HEADERS) $(FLAGS_STAMP)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJECTS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJECTS) -ldl

oracle:
	$(MAKE) -s -C oracle

# phase-timestamp build for tools/trace_select.py (GF_LIB_PATH selects it); never the product
TRACE_OBJDIR := build/obj_trace
TRACE_LIB    := build/libgeoflink_hip_trace.so
TRACE_OBJECTS := $(patsubst $(SRC)/%,$(TRACE_OBJDIR)/%.o,$(SOURCES))
$(TRACE_OBJDIR)/%.o: $(SRC)/% $(HEADERS)
	@mkdir -p $(TRACE_OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DGF_TRACE -x hip -c $< -o $@
$(TRACE_LIB): $(TRACE_OBJECTS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(TRACE_OBJECTS) -ldl
trace: $(TRACE_LIB)

# gfx950 ISA listing for inspection (v_fma_f64 must not appear in the distance paths)
isa: $(LIB)
	/opt/rocm/lib/llvm/bin/clang-offload-bundler --list --type=o --input=$(OBJDIR)/k_knn.hip.o

# Host sanitizer builds: the oracle and the host builds of the product's untrusted-text
# parsers (gf_geojson.hpp / gf_decimal.hpp via tests/native/*.cpp) with AddressSanitizer +
# UndefinedBehaviorSanitizer, and the CPU test suite run against them (the runtimes preloaded
# into python).  Host code only: GPU sanitizers are not available on this pool.
SANFLAGS := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g
ASAN_ORACLE := build/asan/liboracle.so
$(ASAN_ORACLE): oracle/geoflink_oracle.c oracle/cpu_scan.c oracle/geoflink_oracle.h
	@mkdir -p build/asan
	gcc -O1 -fPIC -std=c11 -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function $(SANFLAGS) -pthread -fopenmp \
	    -shared -o $@ oracle/geoflink_oracle.c oracle/cpu_scan.c -lm
asan: $(ASAN_ORACLE)
ASAN_RT := $(shell gcc -print-file-name=libasan.so):$(shell gcc -print-file-name=libubsan.so)
asan-test: asan
	LD_PRELOAD=$(ASAN_RT) ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:allocator_may_return_null=1 \
	UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 GF_ORACLE_LIB=$(abspath $(ASAN_ORACLE)) \
	GF_NATIVE_SANITIZE="$(SANFLAGS)" python -m pytest -x -q -s -m "not gpu" -p no:cacheprovider \
	    tests/test_oracle.py tests/test_csv_core.py tests/test_geojson_core.py tests/test_csv_oracle.py \
	    tests/test_geojson_oracle.py tests/test_windows.py

# Host sanitizers over the PRODUCT's host code: every library source built with
# ASan + UBSan on the host side only (-Xarch_host: the gfx950 device code is the ordinary code --
# GPU sanitizers are not available on this pool), the shim core and the C oracle instrumented the
# same way, and tests/native/asan_driver.c driving the dictionary, the pane ring, the ingest host
# side and the shim's host paths against the oracle.  Built here, run on the GPU box
# (tools/gpu_asan.sh).  clang's ASan runtime throughout (hipcc instruments with it).
CLANG      := /opt/rocm/lib/llvm/bin/clang
HOSTSAN    := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
              -Xarch_host -fno-omit-frame-pointer -Xarch_host -g
CSAN       := -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g
ASAN_GPU   := explibs/asan_gpu
ASAN_OBJS  := $(patsubst $(SRC)/%,$(ASAN_GPU)/obj/%.o,$(SOURCES))
$(ASAN_GPU)/obj/%.o: $(SRC)/% $(HEADERS)
	@mkdir -p $(ASAN_GPU)/obj
	$(HIPCC) $(HIPFLAGS) $(HOSTSAN) -x hip -c $< -o $@
$(ASAN_GPU)/libgeoflink_hip.so: $(ASAN_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(ASAN_OBJS) -ldl
$(ASAN_GPU)/asan_driver: tests/native/asan_driver.c integration/jni/geoflink_shim.c integration/jni/geoflink_shim.h \
                         oracle/geoflink_oracle.c oracle/cpu_scan.c $(ASAN_GPU)/libgeoflink_hip.so
	$(CLANG) -O1 -std=c11 $(CSAN) -ffp-contract=off -fopenmp -Iinclude -I/opt/rocm/include -D__HIP_PLATFORM_AMD__ \
	    tests/native/asan_driver.c integration/jni/geoflink_shim.c oracle/geoflink_oracle.c oracle/cpu_scan.c \
	    -o $@ -L$(ASAN_GPU) -lgeoflink_hip -L/opt/rocm/lib -lamdhip64 -lm -lpthread \
	    -Wl,-rpath,'$$ORIGIN' -Wl,-rpath,/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib
asan-gpu: $(ASAN_GPU)/asan_driver

clean:
	rm -rf build $(LIB) $(SHIM)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle shim clean isa trace asan asan-test asan-gpu
