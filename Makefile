# Build the MI355X (gfx950) evaluator library, the synthetic-segment writer and the CPU oracle.
# Direct hipcc/g++ invocations; `make -j8`.  Outputs land in-tree (git-ignored, shipped to the GPU box).
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
ROCM    ?= /opt/rocm
CXXFLAGS_HOST = -O3 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
HIPFLAGS = -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -munsafe-fp-atomics -Wall -Wno-unused-parameter

SRC     = lakeside_amd/csrc
OBJDIR  = build/obj
LIB     = lakeside_amd/liblakeside_gpu.so
SYNTH   = lakeside_amd/liblakeside_synth.so
RELIB   = lakeside_amd/liblakeside_regex.so
TXLIB   = lakeside_amd/liblakeside_text.so

HOST_SRCS = $(SRC)/numleaf.cpp $(SRC)/exemplar.cpp $(SRC)/jdtoa.cpp $(SRC)/ddsketch.cpp $(SRC)/hll.cpp $(SRC)/regex.cpp $(SRC)/codec.cpp $(SRC)/parquet.cpp $(SRC)/plan.cpp $(SRC)/loader.cpp $(SRC)/engine.cpp $(SRC)/eval.cpp $(SRC)/dims.cpp $(SRC)/comm.cpp $(SRC)/abi.cpp
HOST_OBJS = $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.o,$(HOST_SRCS))
# the fused scan kernels: one unit per (aggregate, kernel family, table mode) so they compile in parallel
SCAN_LEAN  = $(foreach a,sum min max count,$(foreach m,d h,$(OBJDIR)/scan_$(a)_lean_$(m).o))
SCAN_TILES = $(foreach a,sum min max count,$(foreach m,d h,$(OBJDIR)/scan_$(a)_tiles_$(m).o))
HIP_OBJS  = $(OBJDIR)/kernels.o $(OBJDIR)/ex_kernels.o $(SCAN_LEAN) $(SCAN_TILES)
HDRS = $(wildcard $(SRC)/*.hpp) $(SRC)/unicode_tables.inc include/lakeside_gpu.h include/lakeside_regex.h
# device code includes only these (host-only header edits do not rebuild the kernels); lean_kernel.hpp only the
# scan_lean units, scan_kernel.hpp only the scan units
DEV_HDRS = $(SRC)/device_common.hpp $(SRC)/kernels.hpp $(SRC)/layout.hpp $(SRC)/scan_inst.hpp

all: $(LIB) $(SYNTH) $(RELIB) $(TXLIB)

$(OBJDIR)/%.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(CXXFLAGS_HOST) -x c++ -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -c $< -o $@

$(OBJDIR)/%.o: $(SRC)/%.hip $(DEV_HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(SCAN_TILES): $(SRC)/scan_kernel.hpp
$(SCAN_LEAN): $(SRC)/scan_kernel.hpp $(SRC)/lean_kernel.hpp

$(LIB): $(HOST_OBJS) $(HIP_OBJS)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $^ -L$(ROCM)/lib -lrccl -lz -l:libzstd.so.1 -l:liblz4.so.1 -l:libbrotlidec.so.1 -Wl,-rpath,$(ROCM)/lib

# host-only RE2-semantics matcher (CPU differential tests against RE2; the evaluator links regex.cpp itself)
$(RELIB): $(SRC)/regex.cpp $(SRC)/regex_capi.cpp $(SRC)/regex.hpp $(SRC)/unicode_tables.inc include/lakeside_regex.h
	g++ $(CXXFLAGS_HOST) -shared -o $@ $(SRC)/regex.cpp $(SRC)/regex_capi.cpp

# host-only Java 17 number text (CPU differential tests against the oracle's restatement)
$(TXLIB): $(SRC)/jdtoa.cpp $(SRC)/evalutil.hpp include/lakeside_text.h
	g++ $(CXXFLAGS_HOST) -I$(ROCM)/include -D__HIP_PLATFORM_AMD__ -shared -o $@ $(SRC)/jdtoa.cpp

$(SYNTH): tools/synth.cpp $(SRC)/thrift.hpp
	g++ -O3 -std=c++17 -fPIC -shared -pthread -Wall -o $@ tools/synth.cpp

# Kernel ISA for inspection (register use, atomics, load widths)
asm: $(SRC)/kernels.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) --cuda-device-only -S $< -o build/kernels.s
	for a in sum min max count; do for f in lean tiles; do $(HIPCC) $(HIPFLAGS) --cuda-device-only -S $(SRC)/scan_$${a}_$${f}_d.hip -o build/scan_$${a}_$${f}_d.s; done; done

clean:
	rm -rf build $(LIB) $(SYNTH) $(RELIB) $(TXLIB)


.PHONY: all clean asm

# CPU restatement of the evaluator (oracle: test / bench-baseline infrastructure only, never the product path)
CPULIB = oracle/liblkcpu.so
$(CPULIB): oracle/cpu/lkcpu.cpp
	g++ -O3 -std=c++17 -fPIC -fopenmp -shared -Wall -Wextra -Wno-unused-parameter -o $@ $<

all: $(CPULIB)

# Kernel A/B builds (experiments): the library with the scan kernels built under EXP_FLAGS (e.g.
# EXP_FLAGS=-DLK_LEAN_ROWS=4 EXP_NAME=rows4; the scan_lean units only) -> lakeside_amd/exp/liblakeside_gpu_<EXP_NAME>.so,
# selected with LK_LIB_PATH.
EXP_FLAGS ?=
EXP_NAME ?= x
exp: $(HOST_OBJS) $(OBJDIR)/kernels.o $(OBJDIR)/ex_kernels.o $(SCAN_TILES)
	@mkdir -p build/exp/$(EXP_NAME) lakeside_amd/exp
	for a in sum min max count; do for m in d h; do $(HIPCC) $(HIPFLAGS) $(EXP_FLAGS) -c $(SRC)/scan_$${a}_lean_$${m}.hip -o build/exp/$(EXP_NAME)/scan_$${a}_lean_$${m}.o & done; done; wait
	$(HIPCC) -shared --offload-arch=$(ARCH) -o lakeside_amd/exp/liblakeside_gpu_$(EXP_NAME).so $(HOST_OBJS) $(OBJDIR)/kernels.o $(OBJDIR)/ex_kernels.o $(SCAN_TILES) build/exp/$(EXP_NAME)/scan_*.o -L$(ROCM)/lib -lrccl -lz -l:libzstd.so.1 -l:liblz4.so.1 -l:libbrotlidec.so.1 -Wl,-rpath,$(ROCM)/lib
.PHONY: exp

# Host-only loader harness (no HIP): the Parquet walk, dictionary interning and staging copy of lakeside_amd/csrc/
# loader.cpp, plain and under ASan + UBSan / TSan (`make sanitize`, tools/sanitize.sh).
LOADCHK_SRCS = tools/load_check.cpp $(SRC)/loader.cpp $(SRC)/parquet.cpp $(SRC)/codec.cpp $(SRC)/plan.cpp
LOADCHK_DEPS = $(LOADCHK_SRCS) $(SRC)/loader.hpp $(SRC)/segment.hpp $(SRC)/parquet.hpp $(SRC)/codec.hpp $(SRC)/layout.hpp $(SRC)/plan.hpp $(SRC)/thrift.hpp
LOADCHK_FLAGS = -std=c++17 -g -pthread -Wall -Wextra -Wno-unused-parameter
LOADCHK_LIBS = -lz -l:libzstd.so.1 -l:liblz4.so.1 -l:libbrotlidec.so.1
build/load_check: $(LOADCHK_DEPS)
	@mkdir -p build
	g++ -O2 $(LOADCHK_FLAGS) -o $@ $(LOADCHK_SRCS) $(LOADCHK_LIBS)
build/load_check_asan: $(LOADCHK_DEPS)
	@mkdir -p build
	g++ -O1 -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all $(LOADCHK_FLAGS) -o $@ $(LOADCHK_SRCS) $(LOADCHK_LIBS)
build/load_check_tsan: $(LOADCHK_DEPS)
	@mkdir -p build
	g++ -O1 -fsanitize=thread $(LOADCHK_FLAGS) -o $@ $(LOADCHK_SRCS) $(LOADCHK_LIBS)
sanitize: build/load_check build/load_check_asan build/load_check_tsan
	tools/sanitize.sh
.PHONY: sanitize
