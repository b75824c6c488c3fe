# Build the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
# -structurizecfg-skip-uniform-regions: uniform branches stay plain scalar branches (no i1 flow masks in
# SGPR pairs): row kernel 4.70 -> 4.21 ms per 512 1080p pictures (tools/ab_libs2.sh, round 3)
HIPFLAGS ?= -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -shared -Wall -Wno-unused-function -mllvm -structurizecfg-skip-uniform-regions=true
SRC := p265_amd/csrc/p265r.hip
HDR := $(wildcard p265_amd/csrc/*.h) include/p265r.h

CXX ?= g++
FESRC := $(wildcard p265_amd/csrc/fe/*.cpp)
FEHDR := $(wildcard p265_amd/csrc/fe/*.h) include/p265fe.h include/p265r.h

# negative-test builds of the half-CTU publish self-checks (tests/test_a_multirank.py): prep places the
# publish point one job early, with (1) and without (2) prep's own check; and the two A/B phase schedules
# of a pipelined context (tests/test_gpu_parity.py, per-run digests)
CHECKVARIANTS := p265_amd/libp265r_brbroken1.so p265_amd/libp265r_brbroken2.so \
                 p265_amd/libp265r_phaseorder.so p265_amd/libp265r_earlyres.so

all: p265_amd/libp265r.so p265_amd/libp265fe.so p265_amd/libp265probe.so $(CHECKVARIANTS) oracle

p265_amd/libp265r_brbroken%.so: $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -DP265R_BR_BROKEN=$* -o $@ $(SRC)

p265_amd/libp265r_phaseorder.so: $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -DP265R_PHASE_ORDER=1 -o $@ $(SRC)

p265_amd/libp265r_earlyres.so: $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -DP265R_EARLY_RESIDUAL=1 -o $@ $(SRC)

# measurement helper (not the product path): the row kernel's job-loop issue ceiling (bench.py)
p265_amd/libp265probe.so: p265_amd/csrc/issue_probe.hip
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -fPIC -shared -Wall -o $@ $<

# native syntax front-end (host C++, no GPU code)
p265_amd/libp265fe.so: $(FESRC) $(FEHDR)
	$(CXX) -O3 -std=c++17 -fPIC -shared -pthread -Wall -Wextra -Wno-unused-parameter -o $@ $(FESRC)

p265_amd/libp265r.so: $(SRC) $(HDR)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC)

oracle:
	$(MAKE) -C oracle

clean:
	rm -f p265_amd/libp265r.so p265_amd/libp265fe.so p265_amd/libp265probe.so $(CHECKVARIANTS)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# experiment builds: make variant V=name FLAGS="-DX=1"  ->  p265_amd/libp265r_name.so
variant:
	$(HIPCC) $(HIPFLAGS) $(FLAGS) -o p265_amd/libp265r_$(V).so $(SRC)
.PHONY: variant
