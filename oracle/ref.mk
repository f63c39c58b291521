# Builds the REAL reference cKL (the KL parity target) from its
# single source file where it lies under /root/reference, into oracle/_ref/.
# Test infrastructure only: nothing in the product links or runs this.
# cEIG is NOT buildable here (Eigen3 + Spectra absent).
# Flags are the reference Makefile's CXXFLAGS minus the conda include paths
# (Makefile:10-13); no -ffast-math (bit-exact fp32 sums).
REF ?= /root/reference
HERE := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
OUT  := $(HERE)_ref

all: $(OUT)/cKL $(OUT)/cKL_seeded

$(OUT)/cKL: $(REF)/cKL.cpp
	@mkdir -p $(OUT)
	g++ -std=c++17 -O3 -fopenmp $< -o $@

# Random-init runs replayable: the same source with its std::random_device
# seed taken from $EK_REF_SEED (oracle/ref_seed.h, force-included).
$(OUT)/cKL_seeded: $(REF)/cKL.cpp $(HERE)ref_seed.h
	@mkdir -p $(OUT)
	g++ -std=c++17 -O3 -fopenmp -include $(HERE)ref_seed.h $< -o $@

clean:
	rm -rf $(OUT)

.PHONY: all clean
