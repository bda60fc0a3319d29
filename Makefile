# Builds libsyzsig.so (HIP, gfx950 only) in-tree, and the oracle checker.
#   make            -> syzkaller_amd/libsyzsig.so
#   make oracle     -> oracle/liboracle.so (+ oracle/_ref/ref_harness when /root/reference exists)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
JOBS ?= 8
SRC := $(wildcard syzkaller_amd/csrc/*.hip)
OBJDIR ?= build
OBJ := $(patsubst syzkaller_amd/csrc/%.hip,$(OBJDIR)/%.o,$(SRC))
HDR := $(wildcard syzkaller_amd/csrc/*.h) include/syzsig.h
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -munsafe-fp-atomics

LIB := syzkaller_amd/libsyzsig.so

all: $(LIB)

$(OBJDIR)/%.o: syzkaller_amd/csrc/%.hip $(HDR)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJ)

# experiment build: make exp EXP=name EXPFLAGS=-D... -> exp/libsyzsig_name.so (SYZSIG_LIB selects it)
exp:
	@mkdir -p exp/$(EXP)
	$(MAKE) -s -j$(JOBS) LIB=exp/libsyzsig_$(EXP).so OBJDIR=exp/$(EXP) HIPFLAGS="$(HIPFLAGS) $(EXPFLAGS)" exp/libsyzsig_$(EXP).so

oracle:
	$(MAKE) -C oracle all
	@if [ -d /root/reference/executor ]; then $(MAKE) -C oracle ref; fi

clean:
	rm -rf build $(LIB)

.PHONY: all oracle clean exp
