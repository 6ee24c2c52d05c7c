# Build of the MI355X batched SHA-256 library (in-tree, so the .so travels to the GPU box).
#
#   make            -> s3client_amd/lib/libs3hash.so  (C-ABI + lib/hash C++ drop-in + kernels)
#                      oracle/liboracle.so (+ oracle/_ref when /root/reference exists)
#                      tests/cpp binaries (drop-in link tests)
#   make stall      -> tests/cpp/build/libs3hash_stall.so (forced-fault build, GPU tests only)
HIPCC   ?= /opt/rocm/bin/hipcc
CXX     ?= g++
ARCH    ?= gfx950
LIBDIR  := s3client_amd/lib
CSRC    := s3client_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Iinclude

LIB := $(LIBDIR)/libs3hash.so

all: $(LIB) oracle cpptests

# The chain-loop instruction counts bench.py reports, the kernels' code hashes and the
# error-word check are read from the gfx950 code object the linked library ships
# (tools/isa_counts.py -> s3client_amd/kernel_isa_counts.json; disassembly in build/isa).
ISA_DIS := build/isa/libs3hash_gfx950.dis
KSRC := $(CSRC)/capi.hip $(CSRC)/route.hpp $(CSRC)/exp_config.hpp $(CSRC)/sha256_kernels.hip $(CSRC)/sha256_device.hpp $(CSRC)/sha256_skew_rounds.inc $(CSRC)/sha256_producer_simple.inc $(CSRC)/md5_step_asm.inc include/s3hash.h
$(LIBDIR)/capi.o: $(KSRC)
	@mkdir -p $(LIBDIR) build/isa
	cd build/isa && $(HIPCC) $(HIPFLAGS) -save-temps -c -o ../../$@ ../../$<

$(LIBDIR)/lib_hash.o: $(CSRC)/cpu/lib_hash.cpp include/sha256.h include/utility.h include/s3hash.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIBDIR)/lib_md5.o: $(CSRC)/cpu/lib_md5.cpp include/md5.h include/utility.h include/s3hash.h
	@mkdir -p $(LIBDIR)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(LIBDIR)/capi.o $(LIBDIR)/lib_hash.o $(LIBDIR)/lib_md5.o tools/isa_counts.py tools/code_object.py
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(filter %.o,$^) -lpthread
	python3 tools/isa_counts.py $@ s3client_amd/kernel_isa_counts.json $(ISA_DIS)

# Forced-fault build for tests/test_gpu_errors.py: every flag-synchronised producer stops
# publishing after its first step and waits give up after 4,096 polls, so each consumer
# wave's wait times out -- the device error word must fail the call.  Test-only (never the
# product library; loaded through S3H_LIBRARY in a child process).
STALL := tests/cpp/build/libs3hash_stall.so
$(STALL): $(KSRC) $(LIBDIR)/lib_hash.o $(LIBDIR)/lib_md5.o
	@mkdir -p tests/cpp/build
	$(HIPCC) $(HIPFLAGS) -DS3H_EXPERIMENT_BUILD -DS3H_EXP_STALL_PRODUCER=1 -DS3H_EXP_SPIN_LIMIT=4096 -c -o tests/cpp/build/capi_stall.o $(CSRC)/capi.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ tests/cpp/build/capi_stall.o $(LIBDIR)/lib_hash.o $(LIBDIR)/lib_md5.o -lpthread

oracle: $(LIB)
	$(MAKE) -C oracle

CPPTESTS := tests/cpp/build/dropin_test tests/cpp/build/sign_test
cpptests: $(CPPTESTS) apps/build/s3-upload-hash

apps/build/s3-upload-hash: apps/s3_upload_hash.cpp s3client_amd/host/aws_sign.cpp s3client_amd/host/aws_sign.h include/s3hash_batch.hpp $(LIB)
	@mkdir -p apps/build
	$(CXX) -O2 -std=c++17 -pthread -Iinclude -Is3client_amd/host -o $@ $< s3client_amd/host/aws_sign.cpp \
	    -L$(LIBDIR) -ls3hash -Wl,-rpath,'$$ORIGIN/../../$(LIBDIR)'

tests/cpp/build/dropin_test: tests/cpp/dropin_test.cpp include/s3hash_batch.hpp $(LIB)
	@mkdir -p tests/cpp/build
	$(CXX) -O2 -std=c++17 -Iinclude -o $@ $< -L$(LIBDIR) -ls3hash -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

tests/cpp/build/sign_test: tests/cpp/sign_test.cpp s3client_amd/host/aws_sign.cpp s3client_amd/host/aws_sign.h $(LIB)
	@mkdir -p tests/cpp/build
	$(CXX) -O2 -std=c++17 -Iinclude -Is3client_amd/host -o $@ $< s3client_amd/host/aws_sign.cpp \
	    -L$(LIBDIR) -ls3hash -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)'

isa: $(LIBDIR)/capi.o

# the forced-stall library on its own target (test-only; __graft_entry__.build() asks for it)
stall: $(STALL)

# Kernel experiment builds (never the product): make exp TAG=name EXPFLAGS="-DS3H_EXP_..."
# -> tools/exp/libs3hash_<TAG>.so, loaded with S3H_LIBRARY=... python bench.py ...
exp: $(LIBDIR)/lib_hash.o $(LIBDIR)/lib_md5.o
	@mkdir -p tools/exp
	$(HIPCC) $(HIPFLAGS) -DS3H_EXPERIMENT_BUILD $(EXPFLAGS) -c -o tools/exp/capi_$(TAG).o $(CSRC)/capi.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o tools/exp/libs3hash_$(TAG).so tools/exp/capi_$(TAG).o $^ -lpthread

clean:
	rm -rf $(LIBDIR) tests/cpp/build apps/build build
	$(MAKE) -C oracle clean

.PHONY: all oracle cpptests isa stall exp clean
