# Builds the product library (HIP for gfx950 + host C) and the test-only oracle.
#   make            -> uvhttp_amd/lib/libuvhttp_ws_amd.so  +  oracle/_build/libws_oracle.so
ROCM ?= /opt/rocm
HIPCC ?= $(ROCM)/bin/hipcc
CC ?= gcc
ARCH ?= gfx950
BUILD := uvhttp_amd/build
LIB := uvhttp_amd/lib/libuvhttp_ws_amd.so
# the same library built with -DUVWS_TEST_HOOKS -DUVWS_EXPERIMENTS (tests and A/B tools only):
# the batcher's fault-injection hook and the environment switches (UVHTTP_WS_*) the measurements
# and the variant tests use.  The product library reads no environment.
TESTLIB := uvhttp_amd/lib/libuvhttp_ws_amd_testhooks.so
EXP := -DUVWS_EXPERIMENTS

HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Iinclude -Wall -Werror \
            -mcode-object-version=5
CFLAGS := -O2 -DNDEBUG -fPIC -std=gnu11 -Iinclude -Wall -Wextra -Werror

all: $(LIB) $(TESTLIB) oracle ctests probes

$(BUILD)/ws_gpu.o: uvhttp_amd/csrc/ws_gpu.hip include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/tls_gpu.o: uvhttp_amd/csrc/tls_gpu.hip include/uvhttp_tls_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/ws_batcher.o: uvhttp_amd/csrc/ws_batcher.hip include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(BUILD)/ws_batcher_testhooks.o: uvhttp_amd/csrc/ws_batcher.hip include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DUVWS_TEST_HOOKS $(EXP) -c -o $@ $<

$(BUILD)/ws_gpu_exp.o: uvhttp_amd/csrc/ws_gpu.hip include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(EXP) -c -o $@ $<

$(BUILD)/tls_gpu_exp.o: uvhttp_amd/csrc/tls_gpu.hip include/uvhttp_tls_amd.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) $(EXP) -c -o $@ $<

$(BUILD)/ws_host_exp.o: uvhttp_amd/csrc/ws_host.c include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(CC) $(CFLAGS) $(EXP) -c -o $@ $<

$(BUILD)/ws_host.o: uvhttp_amd/csrc/ws_host.c include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(CC) $(CFLAGS) -c -o $@ $<

# host-only C++ (the multi-GPU batcher group): no device code, no HIP headers
$(BUILD)/ws_batcher_group.o: uvhttp_amd/csrc/ws_batcher_group.cpp include/uvhttp_ws_amd.h
	@mkdir -p $(BUILD)
	$(CXX) -O2 -fPIC -std=c++17 -Iinclude -Wall -Wextra -Werror -c -o $@ $<

$(LIB): $(BUILD)/ws_gpu.o $(BUILD)/tls_gpu.o $(BUILD)/ws_batcher.o $(BUILD)/ws_host.o \
        $(BUILD)/ws_batcher_group.o
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

$(TESTLIB): $(BUILD)/ws_gpu_exp.o $(BUILD)/tls_gpu_exp.o $(BUILD)/ws_batcher_testhooks.o $(BUILD)/ws_host_exp.o \
            $(BUILD)/ws_batcher_group.o
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^

oracle:
	$(MAKE) -C oracle

# test programs: the C1 libuv echo harness (against the product library) and the
# ASan/UBSan builds of the host decoder + oracle (tests/c/Makefile)
ctests: $(LIB) oracle
	$(MAKE) -C tests/c

# measurement tools run on the GPU box (PCIe ceilings beside the live-shape e2e)
probes: tools/bin/pcie_probe tools/bin/copy_probe

tools/bin/pcie_probe: tools/pcie_probe.hip
	@mkdir -p tools/bin
	$(HIPCC) --offload-arch=$(ARCH) -O2 -o $@ $<

# host-only (HIP runtime API, no kernels): g++, so the AVX variants can use target attributes
tools/bin/copy_probe: tools/copy_probe.cpp $(BUILD)/ws_host.o
	@mkdir -p tools/bin
	g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -Iinclude -o $@ $^ -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

asm: uvhttp_amd/csrc/ws_gpu.hip uvhttp_amd/csrc/tls_gpu.hip
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -Wno-unused-command-line-argument --cuda-device-only -S -o $(BUILD)/ws_gpu.s uvhttp_amd/csrc/ws_gpu.hip
	$(HIPCC) $(HIPFLAGS) -Wno-unused-command-line-argument --cuda-device-only -S -o $(BUILD)/tls_gpu.s uvhttp_amd/csrc/tls_gpu.hip

clean:
	rm -rf $(BUILD) uvhttp_amd/lib
	$(MAKE) -C oracle clean
	$(MAKE) -C tests/c clean

.PHONY: all oracle ctests probes clean asm
