# Build / test / bench entry points (the reference's per-assignment Makefiles,
# hw/*/programming/Makefile, collapsed into one; `make DEBUG=1` -> -O1 -g as
# there). Native outputs land in 2012-04_stanford_cme213_amd/lib/.
PY ?= python
GPURUN ?= /usr/local/graft/bin/gpurun

ifeq ($(DEBUG),1)
export CME_DEBUG = 1
endif
# TUNE=1: also build csrc/hip_tune/ (the A/B tuning arms) into libcme213_tune.so
ifeq ($(TUNE),1)
export CME_TUNE = 1
endif

.PHONY: all build test test-asan test-gpu bench smoke occupancy clean

all: build

build:
	$(PY) 2012-04_stanford_cme213_amd/_build.py

test: build
	$(PY) -m pytest tests -x -q -m "not gpu"

# CPU backend under AddressSanitizer + UBSan (host code only; the course's
# cuda-memcheck, slides/Lecture06.pdf 2-3): instrumented build in build/asan
test-asan:
	$(PY) scripts/asan_cpu.py

# on a machine with an MI355X
test-gpu: build
	$(PY) -m pytest tests -x -q -m gpu

bench: build
	$(PY) bench.py

smoke: build
	$(PY) -c "import __graft_entry__ as g; g.smoke()"

occupancy: build
	$(PY) -m cme213x occupancy

clean:
	rm -rf build 2012-04_stanford_cme213_amd/lib
