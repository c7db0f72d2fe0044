# Build of the MI355X (gfx950) Reed-Solomon shard codec.
#   make            -> slime_amd/lib/libslime_rs.so (product) + oracle/liboracle.so (test checker)
# hipcc cross-compiles for gfx950 without a GPU present.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Iinclude -Islime_amd/csrc
SRC      := slime_amd/csrc
OBJ      := build/obj
LIB      := slime_amd/lib/libslime_rs.so

OBJS := $(OBJ)/rs_apply.o $(OBJ)/rs_apply_k32.o $(OBJ)/rs_apply_mfma.o $(OBJ)/rs_bytes.o $(OBJ)/rs_bytes_k32.o $(OBJ)/rs_bytes_mfma.o $(OBJ)/gf_codec.o $(OBJ)/host_blit.o $(OBJ)/rs_matrix.o $(OBJ)/host_copy.o $(OBJ)/host_codec.o $(OBJ)/digest.o $(OBJ)/device_alloc.o $(OBJ)/host_pipeline.o $(OBJ)/go_api.o $(OBJ)/object_calls.o $(OBJ)/rs_capi.o
HDRS := $(wildcard $(SRC)/*.hpp) include/slime_rs.h

CXXTEST  := tests/cpp/rs_host_test
CACHETEST := tests/cpp/plan_cache_test
COPYTEST := tests/cpp/copy_pool_test
POOLTEST := tests/cpp/device_pool_test
MFMATEST := tests/cpp/mfma_table_test
DMATEST  := tests/cpp/dma_plan_test
REDOTEST := tests/cpp/redo_list_test
PROXYLOAD := tools/libproxy_load.so

all: $(LIB) oracle $(CXXTEST) $(CACHETEST) $(COPYTEST) $(POOLTEST) $(MFMATEST) $(DMATEST) $(REDOTEST) $(PROXYLOAD)

# Proxy-level load generator over the C-ABI (bench.py host_path.pooled): C++ threads, no GIL.
$(PROXYLOAD): tools/proxy_load.cpp tools/crash_report.hpp include/slime_rs.h $(LIB)
	g++ -std=c++17 -O2 -g -Wall -Wextra -pthread -fPIC -shared -Iinclude -o $@ $< -Lslime_amd/lib -lslime_rs -ldl \
	  -Wl,-rpath,'$$ORIGIN/../slime_amd/lib'

# The matrix-core redo list's counter protocol (redo_list.hpp) emulated with threads, CPU only.
$(REDOTEST): tests/cpp/redo_list_test.cpp $(SRC)/redo_list.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -pthread -I$(SRC) -o $@ tests/cpp/redo_list_test.cpp

# The host pipeline's copy planning and extent checks (dma_plan.hpp), CPU only.
$(DMATEST): tests/cpp/dma_plan_test.cpp $(SRC)/dma_plan.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -I$(SRC) -o $@ tests/cpp/dma_plan_test.cpp

# The matrix-core kernel's int8-limb arithmetic emulated on its table (mfma_table.hpp), CPU only.
$(MFMATEST): tests/cpp/mfma_table_test.cpp $(SRC)/mfma_table.hpp $(SRC)/gfp.hpp $(SRC)/gfp_host.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -I$(SRC) -o $@ tests/cpp/mfma_table_test.cpp

# Device routing of host calls (device_pool.hpp) with a fixed device count, CPU only.
$(POOLTEST): tests/cpp/device_pool_test.cpp $(SRC)/device_pool.hpp $(SRC)/plan_cache.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -pthread -I$(SRC) -o $@ tests/cpp/device_pool_test.cpp

# The host copy pool under concurrent callers, CPU only.
$(COPYTEST): tests/cpp/copy_pool_test.cpp $(SRC)/host_copy.cpp $(SRC)/host_copy.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -pthread -I$(SRC) -o $@ tests/cpp/copy_pool_test.cpp $(SRC)/host_copy.cpp

# The plan cache (plan_cache.hpp) over the product's host matrix code, CPU only.
$(CACHETEST): tests/cpp/plan_cache_test.cpp $(SRC)/plan_cache.hpp $(SRC)/rs_matrix.cpp $(SRC)/rs_matrix.hpp
	g++ -std=c++17 -O2 -Wall -Wextra -pthread -I$(SRC) -o $@ tests/cpp/plan_cache_test.cpp $(SRC)/rs_matrix.cpp

# C++ host mirror of the Go API (include/slime_rs.hpp) and its parity tests.
$(CXXTEST): tests/cpp/rs_host_test.cpp include/slime_rs.hpp include/slime_rs.h $(LIB)
	g++ -std=c++17 -O2 -Wall -Wextra -pthread -Iinclude -o $@ $< -Lslime_amd/lib -lslime_rs \
	  -Wl,-rpath,'$$ORIGIN/../../slime_amd/lib'

$(OBJ)/%.o: $(SRC)/%.hip $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJ)/%.o: $(SRC)/%.cpp $(HDRS) | $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS) -Wl,-soname,libslime_rs.so -Wl,--no-undefined -lpthread

$(OBJ):
	@mkdir -p $@

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(PROXYLOAD) $(CXXTEST) $(CACHETEST) $(COPYTEST) $(POOLTEST) $(MFMATEST) $(DMATEST) $(REDOTEST)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# Host-call latency through the C-ABI alone (tools only): make tools/latency_c
tools/latency_c: tools/latency_c.cpp include/slime_rs.h $(LIB)
	g++ -std=c++17 -O2 -Wall -Wextra -Iinclude -o $@ $< -Lslime_amd/lib -lslime_rs -Wl,-rpath,'$$ORIGIN/../slime_amd/lib'

# Micro-benchmarks (tools only): make ubench
ubench: tools/libubench.so
tools/libubench.so: tools/ubench.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: ubench

# Stamped twin of the product's queue apply launch (tools only): make tools/libc2stamps.so
tools/libc2stamps.so: tools/c2_stamps.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

# Apply-kernel variant harness (tools only): make applyvar
applyvar: tools/libapplyvar.so
tools/libapplyvar.so: tools/apply_variants.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: applyvar

# Byte-domain kernel variant harness (tools only): make bytesvar
bytesvar: tools/libbytesvar.so
tools/libbytesvar.so: tools/bytes_variants.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: bytesvar

# Byte encode first-pass unroll / unit variants (tools only): make bqvar
bqvar: tools/libbqvar.so
tools/libbqvar.so: tools/bytes_queue_variants.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: bqvar

# Byte encode second pass: re-encode vs top-bit correction (tools only): make topbits
topbits: tools/libtopbits.so
tools/libtopbits.so: tools/topbits_fix.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: topbits

# Hash throughput probe for §8(f3) (tools only): make hashprobe
hashprobe: tools/libhashprobe.so
tools/libhashprobe.so: tools/hash_probe.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: hashprobe

# Placement-mode probe (tools only): make placeprobe
placeprobe: tools/libplaceprobe.so
tools/libplaceprobe.so: tools/placement_probe.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: placeprobe

# Physical-placement probe (tools only): make tools/vmm_probe
tools/vmm_probe: tools/vmm_probe.hip include/slime_rs.h $(LIB)
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -Iinclude -o $@ $< -Lslime_amd/lib -lslime_rs \
	  -Wl,-rpath,'$$ORIGIN/../slime_amd/lib'

# Matrix-core apply variants at five K steps (tools only): make widevar
widevar: tools/libwidevar.so
tools/libwidevar.so: tools/wide_variants.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<
.PHONY: widevar
