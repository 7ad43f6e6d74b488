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
             $(wildcard csrc/kafka/*.cpp) $(wildcard csrc/bindings/*.cpp)
HIP_OBJ   := $(patsubst csrc/%.hip,$(OBJ)/%.o,$(HIP_SRC))
CXX_OBJ   := $(patsubst csrc/%.cpp,$(OBJ)/%.o,$(CXX_SRC))
HDRS      := $(wildcard csrc/include/gale/*.h) $(wildcard csrc/kernels/*.cuh) \
             $(wildcard csrc/runtime/*.h) $(wildcard csrc/codec/*.h) $(wildcard csrc/kafka/*.h)

all: gale/_C.so

$(OBJ)/%.o: csrc/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIP_FLAGS) -c $< -o $@

$(OBJ)/%.o: csrc/%.cpp $(HDRS)
	@mkdir -p $(dir $@)
	$(CXX) $(CXX_FLAGS) -c $< -o $@

gale/_C.so: $(HIP_OBJ) $(CXX_OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -L$(ROCM)/lib -lamdhip64 -lrocprofiler-sdk-roctx -pthread \
	    -Wl,-rpath,$(ROCM)/lib

clean:
	rm -rf build gale/_C.so

.PHONY: all clean
