# Build of the MI355X-native GraphBLAS execution layer.
#   make            libgx.so (HIP, gfx950) + bin/exe/* (Graphalytics executables) + oracle
#   make lib        libgx.so only
#   make oracle     oracle/liboracle.so (CPU restatement, test infrastructure only)
# The reference's own CMake build (src/main/c/CMakeLists.txt) is not used: it needs
# SuiteSparse:GraphBLAS/LAGraph, which this layer replaces.

PKG      := ldbc_graphalytics_platforms_graphblas_amd
CSRC     := $(PKG)/csrc
EXESRC   := $(PKG)/exe
BUILD    := build
ARCH     ?= gfx950
HIPCC    ?= /opt/rocm/bin/hipcc
CXX      ?= g++
CC       ?= gcc

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wall -Wno-unused-result
CXXFLAGS := -O3 -std=c++17 -fPIC -fopenmp -Iinclude -I$(CSRC) -Wall -Wextra
LIBGX    := $(PKG)/libgx.so

HIP_SRCS := $(wildcard $(CSRC)/*.hip)
HOST_SRCS := $(wildcard $(CSRC)/*.cpp)
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(BUILD)/%.hip.o,$(HIP_SRCS))
HOST_OBJS := $(patsubst $(CSRC)/%.cpp,$(BUILD)/%.o,$(HOST_SRCS))

EXES := bfs pr sssp wcc cdlp lcc converter
EXE_BINS := $(addprefix bin/exe/,$(EXES))

.PHONY: all lib exe oracle clean probe
all: lib exe oracle
lib: $(LIBGX)
exe: $(EXE_BINS)
oracle: oracle/liboracle.so

$(BUILD):
	mkdir -p $(BUILD)

$(BUILD)/%.hip.o: $(CSRC)/%.hip $(wildcard $(CSRC)/*.h) include/gx.h | $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/%.o: $(CSRC)/%.cpp $(wildcard $(CSRC)/*.h) include/gx.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIBGX): $(HIP_OBJS) $(HOST_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lgomp -ldl -Wl,-soname,libgx.so

$(BUILD)/exe_common.o: $(EXESRC)/common.cpp $(EXESRC)/common.h include/gx.h | $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

bin/exe/%: $(EXESRC)/%.cpp $(BUILD)/exe_common.o $(LIBGX) $(EXESRC)/common.h
	@mkdir -p bin/exe
	$(CXX) $(CXXFLAGS) -o $@ $< $(BUILD)/exe_common.o -L$(PKG) -lgx \
	    -Wl,-rpath,'$$ORIGIN/../../$(PKG)'

oracle/liboracle.so: oracle/gx_oracle.c
	$(CC) -O3 -fPIC -shared -fopenmp -Wall -Wextra -o $@ $<

clean:
	rm -rf $(BUILD) $(LIBGX) $(EXE_BINS) oracle/liboracle.so

# Diagnostic build (not the product): libgx with the PageRank timing probes of
# gx_pr_sorted.hip (GX_PR_PROBE=1..7, wrong results by design), for tools/pr_probe.sh
# (tools/ travels to the GPU box; build/ does not).
PROBE_DIR := $(BUILD)/probe
probe: tools/probe/libgx.so
$(PROBE_DIR)/gx_pr_sorted.hip.o: $(CSRC)/gx_pr_sorted.hip $(wildcard $(CSRC)/*.h) include/gx.h | $(BUILD)
	mkdir -p $(PROBE_DIR)
	$(HIPCC) $(HIPFLAGS) -DGX_PR_PROBES -c $< -o $@
tools/probe/libgx.so: $(filter-out $(BUILD)/gx_pr_sorted.hip.o,$(HIP_OBJS)) $(PROBE_DIR)/gx_pr_sorted.hip.o $(HOST_OBJS)
	@mkdir -p tools/probe
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -lgomp -ldl -Wl,-soname,libgx.so
