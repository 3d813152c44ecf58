# Convenience targets (reference counterpart: Makefile:1-153, `make test`).
PY ?= python
GPURUN ?= /usr/local/graft/bin/gpurun

.PHONY: build cmake test gputest bench clean

build:            ## in-tree build of _hf2d, bin/hf2d, bin/hf2d_cpu (ninja, hipcc gfx950)
	$(PY) -c "import __graft_entry__ as g; g.build()"

cmake:            ## the same targets through CMake, installed into the package
	cmake -S . -B build/cmake -G Ninja && cmake --build build/cmake -j8 && cmake --install build/cmake

test: build       ## CPU suite (reference decks, steppers, distributed gloo, CLI)
	$(PY) -m pytest tests -x -q -m "not gpu"

gputest: build    ## GPU suite on an MI355X box
	$(GPURUN) --timeout 900 -- 'bash tools/gpu_suite.sh all'

bench: build      ## headline benchmark, one GPU
	$(PY) bench.py

clean:
	rm -rf build
