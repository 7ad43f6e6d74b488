# gale native build: hand-written gfx950 HIP kernels + C++ host runtime -> gale/_C.so
# (in-tree, so the built library travels with the repo snapshot to the GPU box).
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
CXX       ?= g++
ARCH      ?= gfx950
PYTHON    ?= python3
PY_INC    := $(shell $(PYTHON) -c "import sysconfig;print(sysconfig.get_paths()['include'])")
PYBIND_INC:= $(shell $(PYTHON) -c "import pybind11;print(pybind11.get_include())")
OBJ       := build/obj

HIP_FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Icsrc/include -Icsrc/kernels \
             -Wno-unused-result
CXX_FLAGS := -O3 -fPIC -std=c++17 -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -Icsrc/include \
             -I$(PY_INC) -I$(PYBIND_INC) -mavx2 -mfma -msse4.2 -mpclmul -mbmi2 -pthread \
             -fvisibility=hidden -Wall -Wno-unused-function -Wno-unused-result

HIP_SRC   := $(wildcard csrc/kernels/*.hip)
CXX_SRC   := $(wildcard csrc/runtime/*.cpp) $(wildcard csrc/codec/*.cpp) \
             $(wildcard csrc/kafka/*.cpp) $(wildcard csrc/comm/*.cpp) $(wildcard csrc/bindings/*.cpp)
HIP_OBJ   := $(patsubst csrc/%.hip,$(OBJ)/%.o,$(HIP_SRC))
CXX_OBJ   := $(patsubst csrc/%.cpp,$(OBJ)/%.o,$(CXX_SRC))
HDRS      := $(wildcard csrc/include/gale/*.h) $(wildcard csrc/kernels/*.cuh) \
             $(wildcard csrc/runtime/*.h) $(wildcard csrc/codec/*.h) $(wildcard csrc/kafka/*.h) \
             $(wildcard csrc/comm/*.h)

all: gale/_C.so

$(OBJ)/%.o: csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIP_FLAGS) -c $< -o $@

$(OBJ)/%.o: csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXX_FLAGS) -c $< -o $@

gale/_C.so: $(HIP_OBJ) $(CXX_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L$(ROCM)/lib -lamdhip64 -lrccl -lrocprofiler-sdk-roctx -lz -ldl -pthread \
	    -Wl,-rpath,$(ROCM)/lib

clean:
	rm -rf build gale/_C.so

.PHONY: all clean

# ---- host-pipeline sanitizer builds: engine + Kafka client/broker + codec with
# CPU stub replicas under ThreadSanitizer / AddressSanitizer. Host code only (no GPU code is
# linked; GPU sanitizers are not available on this pool).
SAN_SRC   := csrc/tests/engine_stress.cpp csrc/runtime/engine.cpp csrc/runtime/replica.cpp \
             csrc/runtime/pinned_pool.cpp csrc/runtime/trace.cpp csrc/codec/json_codec.cpp \
             csrc/codec/text_pack.cpp csrc/codec/java8_float.cpp \
             $(wildcard csrc/kafka/*.cpp)
SAN_FLAGS := -O1 -g -fno-omit-frame-pointer -std=c++17 -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include \
             -Icsrc/include -mavx2 -mfma -msse4.2 -mpclmul -mbmi2 -pthread
SAN_LIBS  := -L$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -lz -ldl -Wl,-rpath,$(ROCM)/lib
# LLVM's sanitizer runtimes (ROCm's clang): gcc-11's libtsan does not intercept
# pthread_cond_clockwait, which libstdc++'s condition_variable uses, and reports false races
SAN_CXX   ?= $(ROCM)/lib/llvm/bin/clang++

build/tsan/engine_stress: $(SAN_SRC) $(HDRS)
	@mkdir -p $(dir $@)
	$(SAN_CXX) $(SAN_FLAGS) -fsanitize=thread $(SAN_SRC) -o $@ $(SAN_LIBS)

build/asan/engine_stress: $(SAN_SRC) $(HDRS)
	@mkdir -p $(dir $@)
	$(SAN_CXX) $(SAN_FLAGS) -fsanitize=address,undefined -fno-sanitize-recover=undefined $(SAN_SRC) -o $@ $(SAN_LIBS)

tsan: build/tsan/engine_stress
	TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1" ./build/tsan/engine_stress 1500

asan: build/asan/engine_stress
	ASAN_OPTIONS="detect_leaks=1" ./build/asan/engine_stress 2000

.PHONY: tsan asan

# host codec micro-benchmark (CRC32C + envelope scan GB/s per core)
build/host_bench: csrc/tests/host_bench.cpp csrc/codec/json_codec.cpp csrc/kafka/wire.cpp $(HDRS)
	@mkdir -p build
	$(CXX) -O3 -std=c++17 -mavx2 -mfma -msse4.2 -mpclmul -mbmi2 -Icsrc/include \
	    csrc/tests/host_bench.cpp csrc/codec/json_codec.cpp csrc/kafka/wire.cpp -o $@

# DRAM antagonist for the host-projection test (tools/dram_antagonist.cpp); outside build/ so it
# travels to the GPU box (build/ is gpurun-ignored)
tools/bin/dram_antagonist: tools/dram_antagonist.cpp
	@mkdir -p tools/bin
	$(CXX) -O2 -std=c++17 -mavx2 -pthread $< -o $@

antagonist: tools/bin/dram_antagonist
.PHONY: antagonist
