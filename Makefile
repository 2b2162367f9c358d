# Build of the MI355X-native CPD engine (replaces the reference's install.sh,
# which ran `make fast` in the warthog submodule and copied make_cpd_auto,
# gen_distribute_conf and fifo_auto into ./bin — install.sh:3-21).
#
#   make            libcpd.so + bin/* + oracle (checker)
#   make lib        distributed-oracle-search_amd/libcpd.so
#   make bins       bin/make_cpd_auto bin/fifo_auto bin/gen_distribute_conf bin/gen_synth
#   make oracle     oracle/libcpd_oracle.so (test infrastructure only)

ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
CC        ?= gcc
ARCH      ?= gfx950
PKG       := distributed-oracle-search_amd
SRC       := $(PKG)/csrc
BLD       := $(PKG)/build
LIB       := $(PKG)/libcpd.so
ORACLE    := oracle/libcpd_oracle.so

CXXFLAGS  := -O3 -std=c++17 -fPIC -fopenmp -Wall -Wextra -Wno-unused-parameter \
             -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -Iinclude -I$(SRC)
HIPFLAGS  := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Iinclude -I$(SRC) \
             -Wall -Wno-unused-parameter
LDLIBS    := -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

HOST_OBJS := $(BLD)/host_util.o $(BLD)/ch.o $(BLD)/ch_gpu.o $(BLD)/plan.o $(BLD)/cpd_gpu.o $(BLD)/cpd_io.o
DEV_OBJS  := $(BLD)/cpd_kernels.o $(BLD)/ch_kernels.o
TOOLS     := make_cpd_auto fifo_auto gen_distribute_conf gen_synth
BINS      := $(addprefix bin/,$(TOOLS))
HDRS      := include/cpd_api.h $(SRC)/cpd_internal.hpp $(SRC)/cpd_kernels.hpp $(SRC)/cpd_io.hpp \
             $(SRC)/ch_kernels.hpp

# Build provenance: sha256 over the library's and tools' sources (sorted by
# path, contents concatenated — cpd.src_sha() recomputes it from the shipped
# tree), embedded in cpd_version() so a run can prove which sources its
# libcpd.so was built from.
PROV_SRCS := $(sort $(wildcard include/*.h $(SRC)/*.cpp $(SRC)/*.hpp $(SRC)/*.hip \
                               $(PKG)/tools/*.cpp $(PKG)/tools/*.hpp))
SRC_SHA    = $(shell cat $(PROV_SRCS) | sha256sum | cut -c1-16)

.PHONY: all lib bins oracle clean FORCE
all: lib bins oracle
lib: $(LIB)
bins: $(BINS)
oracle: $(ORACLE)

$(BLD):
	mkdir -p $(BLD) bin

$(BLD)/%.o: $(SRC)/%.cpp $(HDRS) | $(BLD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

# rewritten only when the hash changes, so an unchanged tree rebuilds nothing
$(BLD)/src_sha.h: FORCE | $(BLD)
	@echo '#define CPD_SRC_SHA "$(SRC_SHA)"' > $@.tmp; \
	 if cmp -s $@.tmp $@; then rm -f $@.tmp; else mv $@.tmp $@; fi

$(BLD)/host_util.o: $(SRC)/host_util.cpp $(HDRS) $(BLD)/src_sha.h | $(BLD)
	$(CXX) $(CXXFLAGS) -I$(BLD) -c $< -o $@


$(BLD)/cpd_kernels.o: $(SRC)/cpd_kernels.hip $(SRC)/cpd_kernels.hpp | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BLD)/ch_kernels.o: $(SRC)/ch_kernels.hip $(SRC)/ch_kernels.hpp | $(BLD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HOST_OBJS) $(DEV_OBJS)
	$(CXX) -shared -fopenmp -o $@ $^ $(LDLIBS)

bin/%: $(PKG)/tools/%.cpp $(LIB) $(HDRS) | $(BLD)
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(PKG) -lcpd -Wl,-rpath,'$$ORIGIN/../$(PKG)' $(LDLIBS)

$(ORACLE): oracle/cpd_oracle.c
	$(CC) -O2 -std=c11 -fPIC -fopenmp -shared -Wall -o $@ $<

clean:
	rm -rf $(BLD) $(LIB) $(BINS) $(ORACLE)
