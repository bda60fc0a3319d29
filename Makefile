# Builds libsyzsig.so (HIP, gfx950 only) in-tree, and the oracle checker.
#   make            -> syzkaller_amd/libsyzsig.so
#   make oracle     -> oracle/liboracle.so (+ oracle/_ref/ref_harness when /root/reference exists)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8
SRC := $(wildcard syzkaller_amd/csrc/*.hip)
OBJ := $(patsubst syzkaller_amd/csrc/%.hip,build/%.o,$(SRC))
HDR := $(wildcard syzkaller_amd/csrc/*.h) include/syzsig.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics

LIB := syzkaller_amd/libsyzsig.so

all: $(LIB)

build/%.o: syzkaller_amd/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

oracle:
	$(MAKE) -C oracle all
	@if [ -d /root/reference/executor ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf build $(LIB)

.PHONY: all oracle clean
