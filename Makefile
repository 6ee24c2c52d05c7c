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
OBJDIR  := $(LIBDIR)/obj
CSRC    := s3client_amd/csrc
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -fno-slp-vectorize -MMD -MP
CXXFLAGS := -O3 -std=c++17 -fPIC -Wall -Iinclude -MMD -MP
# host translation units: plain C++ against the HIP runtime API (no device code)
HOSTFLAGS := -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter -D__HIP_PLATFORM_AMD__ \
             -I/opt/rocm/include -Iinclude -MMD -MP

LIB := $(LIBDIR)/libs3hash.so

all: $(LIB) oracle cpptests

# libs3hash.so = one device unit (launch.hip: the kernels of sha256_kernels.hip and their
# launches) + host units by concern (internal.hpp lists them) + the CPU drop-in.
HOST_UNITS := status topology plan pinned host_path stream route_plan route
HOST_OBJS := $(HOST_UNITS:%=$(OBJDIR)/%.o)
CPU_OBJS := $(OBJDIR)/lib_hash.o $(OBJDIR)/lib_md5.o
KERNEL_OBJ := $(OBJDIR)/launch.o

# The chain-loop instruction counts bench.py reports, the kernels' code hashes and the
# error-word check are read from the gfx950 code object the linked library ships
# (tools/isa_counts.py -> s3client_amd/kernel_isa_counts.json; disassembly in build/isa).
ISA_DIS := build/isa/libs3hash_gfx950.dis
# (explicit prerequisites: the -MMD file is written from build/isa, so its relative paths do not
# resolve from the repo root)
KERNEL_SRCS := $(CSRC)/launch.hip $(CSRC)/sha256_kernels.hip $(wildcard $(CSRC)/*.inc) \
               $(CSRC)/sha256_device.hpp $(CSRC)/kernel_abi.hpp $(CSRC)/exp_config.hpp $(CSRC)/internal.hpp
$(KERNEL_OBJ): $(KERNEL_SRCS)
	@mkdir -p $(OBJDIR) build/isa
	cd build/isa && $(HIPCC) $(HIPFLAGS) -MF ../../$(@:.o=.d) -save-temps -c -o ../../$@ ../../$(CSRC)/launch.hip

$(OBJDIR)/%.o: $(CSRC)/%.cpp
	@mkdir -p $(OBJDIR)
	$(CXX) $(HOSTFLAGS) -c -o $@ $<

$(OBJDIR)/%.o: $(CSRC)/cpu/%.cpp
	@mkdir -p $(OBJDIR)
	$(CXX) $(CXXFLAGS) -c -o $@ $<

$(LIB): $(KERNEL_OBJ) $(HOST_OBJS) $(CPU_OBJS) tools/isa_counts.py tools/code_object.py
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(filter %.o,$^) -lpthread
	python3 tools/isa_counts.py $@ s3client_amd/kernel_isa_counts.json $(ISA_DIS)

-include $(wildcard $(OBJDIR)/*.d)

# Forced-fault build for tests/test_gpu_errors.py: every flag-synchronised producer stops
# publishing after its first step and waits give up after 4,096 polls, so each consumer
# wave's wait times out -- the device error word must fail the call.  Test-only (never the
# product library; loaded through S3H_LIBRARY in a child process).  The switches are device
# code only: the product's host units are linked unchanged.
STALL := tests/cpp/build/libs3hash_stall.so
$(STALL): $(CSRC)/launch.hip $(KERNEL_OBJ) $(HOST_OBJS) $(CPU_OBJS)
	@mkdir -p tests/cpp/build
	$(HIPCC) $(HIPFLAGS) -MF tests/cpp/build/launch_stall.d -DS3H_EXPERIMENT_BUILD -DS3H_EXP_STALL_PRODUCER=1 -DS3H_EXP_SPIN_LIMIT=4096 -c -o tests/cpp/build/launch_stall.o $(CSRC)/launch.hip
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ tests/cpp/build/launch_stall.o $(HOST_OBJS) $(CPU_OBJS) -lpthread

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

isa: $(KERNEL_OBJ)

# the forced-stall library on its own target (test-only; __graft_entry__.build() asks for it)
stall: $(STALL)

# Kernel / plan experiment builds (never the product): make exp TAG=name EXPFLAGS="-DS3H_EXP_..."
# -> tools/exp/libs3hash_<TAG>.so (every unit rebuilt with the flags: some change host choices),
# loaded with S3H_LIBRARY=... python bench.py ...
EXPDIR = tools/exp/$(TAG)
exp:
	@mkdir -p $(EXPDIR)
	$(HIPCC) $(HIPFLAGS) -DS3H_EXPERIMENT_BUILD $(EXPFLAGS) -c -o $(EXPDIR)/launch.o $(CSRC)/launch.hip
	for u in $(HOST_UNITS); do $(CXX) $(HOSTFLAGS) -DS3H_EXPERIMENT_BUILD $(EXPFLAGS) -c -o $(EXPDIR)/$$u.o $(CSRC)/$$u.cpp || exit 1; done
	$(CXX) $(CXXFLAGS) -c -o $(EXPDIR)/lib_hash.o $(CSRC)/cpu/lib_hash.cpp
	$(CXX) $(CXXFLAGS) -c -o $(EXPDIR)/lib_md5.o $(CSRC)/cpu/lib_md5.cpp
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o tools/exp/libs3hash_$(TAG).so $(EXPDIR)/*.o -lpthread

clean:
	rm -rf $(LIBDIR) tests/cpp/build apps/build build
	$(MAKE) -C oracle clean

.PHONY: all oracle cpptests isa stall exp clean
