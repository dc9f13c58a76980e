# MI355X (gfx950) build of the drop-in libwhisper.so (C ABI of include/whisper.h + owk.h).
#
#   make            -> open-whisper-kit_amd/lib/libwhisper.so
#   make oracle     -> oracle/_ref/libwhisper_ref.so (reference CPU path; test infrastructure)
#
# hipcc cross-compiles for gfx950 without a GPU. -ffp-contract=off keeps every
# elementwise f32 op a single rounding like the reference's separate ggml ops
# (fused multiply-adds are written explicitly where the reference fuses).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
JOBS     ?= 8
PKG      := open-whisper-kit_amd
SRC      := $(PKG)/csrc
OBJDIR   := $(PKG)/build
LIB      := $(PKG)/lib/libwhisper.so
SFLIB    := $(PKG)/lib/libsortformer.so

FLAGS    := -O3 -g -std=c++17 -fPIC -ffp-contract=off --offload-arch=$(ARCH) -Iinclude -I$(SRC) \
            -DWHISPER_SHARED -DWHISPER_BUILD -Wall -Wno-unused-function -Wno-unused-variable

HIP_SRCS := $(wildcard $(SRC)/*.hip)
CPP_SRCS := $(wildcard $(SRC)/*.cpp)
ALL_OBJS := $(patsubst $(SRC)/%.hip,$(OBJDIR)/%.hip.o,$(HIP_SRCS)) \
            $(patsubst $(SRC)/%.cpp,$(OBJDIR)/%.cpp.o,$(CPP_SRCS))
# libsortformer.so: the SortFormer C ABI (include/sortformer.h) + the shared GEMM/LayerNorm kernels
SF_ONLY  := $(OBJDIR)/sortformer.cpp.o $(OBJDIR)/k_sortformer.hip.o
OBJS     := $(filter-out $(SF_ONLY),$(ALL_OBJS))
SF_OBJS  := $(SF_ONLY) $(OBJDIR)/k_gemm.hip.o $(OBJDIR)/k_misc.hip.o $(OBJDIR)/kquant.cpp.o
HDRS     := $(wildcard $(SRC)/*.h) $(wildcard include/*.h)

all: $(LIB) $(SFLIB)

$(SFLIB): $(SF_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(SF_OBJS) -Wl,--no-undefined -Wl,-soname,libsortformer.so

$(LIB): $(OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -o $@ $(OBJS) -rdynamic -Wl,--no-undefined -Wl,-soname,libwhisper.so

$(OBJDIR)/%.hip.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -c $< -o $@

$(OBJDIR)/%.cpp.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(FLAGS) -x hip -c $< -o $@

SELFTEST := $(PKG)/lib/owk_selftest

$(SELFTEST): tools/owk_selftest.cpp $(LIB)
	g++ -O1 -g -std=c++17 -Iinclude -o $@ $< -L$(PKG)/lib -lwhisper -Wl,-rpath,'$$ORIGIN'

selftest: $(SELFTEST)

oracle:
	$(MAKE) -C oracle/ref -j$(JOBS)

# The reference's own C/C++ callers, compiled UNCHANGED from /root/reference against
# include/ and linked to our libraries (the drop-in claim of INTEGRATION.md). Built here
# (this container has the sources); the binaries travel to the GPU box in lib/callers/.
REF      ?= /root/reference
CALLERS  := $(PKG)/lib/callers
EXCOMMON := $(REF)/examples/common.cpp $(REF)/examples/common-whisper.cpp $(REF)/examples/grammar-parser.cpp
CALLFLAGS := -O2 -std=c++17 -w -Iinclude -I$(REF)/examples

callers: $(CALLERS)/whisper-cli $(CALLERS)/whisper-bench $(CALLERS)/sortformer-diarize $(CALLERS)/test-streaming-api

$(CALLERS)/whisper-cli: $(REF)/examples/cli/cli.cpp $(EXCOMMON) $(LIB) $(HDRS)
	@mkdir -p $(CALLERS)
	g++ $(CALLFLAGS) $< $(EXCOMMON) -o $@ -L$(PKG)/lib -lwhisper -Wl,-rpath,'$$ORIGIN/..'

$(CALLERS)/whisper-bench: $(REF)/examples/bench/bench.cpp $(EXCOMMON) $(LIB) $(HDRS)
	@mkdir -p $(CALLERS)
	g++ $(CALLFLAGS) $< $(EXCOMMON) -o $@ -L$(PKG)/lib -lwhisper -Wl,-rpath,'$$ORIGIN/..'

$(CALLERS)/sortformer-diarize: $(REF)/streaming-sortformer/src/sortformer-cli.cpp $(SFLIB) $(HDRS)
	@mkdir -p $(CALLERS)
	g++ $(CALLFLAGS) $< -o $@ -L$(PKG)/lib -lsortformer -Wl,-rpath,'$$ORIGIN/..'

$(CALLERS)/test-streaming-api: $(REF)/streaming-sortformer/src/test-streaming-api.cpp $(SFLIB) $(HDRS)
	@mkdir -p $(CALLERS)
	g++ $(CALLFLAGS) $< -o $@ -L$(PKG)/lib -lsortformer -Wl,-rpath,'$$ORIGIN/..'

# Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of both libraries (the reference's
# WHISPER_SANITIZE_ADDRESS / _UNDEFINED, ref CMakeLists.txt:74-76, 99-101). Only host code is
# instrumented (each -fsanitize= after -Xarch_host; device code objects are unchanged), so the
# libraries load and run their host paths on this GPU-less container: tokenizer, model/GGUF header
# parsing, GBNF grammar, aligner, RTTM, DTW, k-quant expansion, VAD segments, KV-cell allocator.
#   make sanitize        -> open-whisper-kit_amd/lib/san/{libwhisper,libsortformer}.so
#   make sanitize-test   -> the CPU tests of those paths against them (tools/sanitize_tests.sh)
SANDIR   := $(PKG)/build_san
SANLIB   := $(PKG)/lib/san
SANFLAGS := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
            -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize=vptr
SAN_OBJS_ALL := $(patsubst $(SRC)/%.hip,$(SANDIR)/%.hip.o,$(HIP_SRCS)) $(patsubst $(SRC)/%.cpp,$(SANDIR)/%.cpp.o,$(CPP_SRCS))
SAN_SF_ONLY  := $(SANDIR)/sortformer.cpp.o $(SANDIR)/k_sortformer.hip.o
SAN_OBJS     := $(filter-out $(SAN_SF_ONLY),$(SAN_OBJS_ALL))
SAN_SF_OBJS  := $(SAN_SF_ONLY) $(SANDIR)/k_gemm.hip.o $(SANDIR)/k_misc.hip.o $(SANDIR)/kquant.cpp.o

sanitize: $(SANLIB)/libwhisper.so $(SANLIB)/libsortformer.so

$(SANLIB)/libwhisper.so: $(SAN_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -shared-libasan -fsanitize=address,undefined -o $@ $(SAN_OBJS) -rdynamic \
	    -Wl,-soname,libwhisper.so

$(SANLIB)/libsortformer.so: $(SAN_SF_OBJS)
	@mkdir -p $(dir $@)
	$(HIPCC) -shared --offload-arch=$(ARCH) -shared-libasan -fsanitize=address,undefined -o $@ $(SAN_SF_OBJS) \
	    -Wl,-soname,libsortformer.so

$(SANDIR)/%.hip.o: $(SRC)/%.hip $(HDRS)
	@mkdir -p $(SANDIR)
	$(HIPCC) $(FLAGS) $(SANFLAGS) -c $< -o $@

$(SANDIR)/%.cpp.o: $(SRC)/%.cpp $(HDRS)
	@mkdir -p $(SANDIR)
	$(HIPCC) $(FLAGS) $(SANFLAGS) -x hip -c $< -o $@

sanitize-test: sanitize
	bash tools/sanitize_tests.sh

clean:
	rm -rf $(OBJDIR) $(SANDIR) $(PKG)/lib

.PHONY: all clean oracle selftest callers sanitize sanitize-test
