# Build / test / package entry points (reference analogue: Makefile:52-144).
include versions.mk

BUILD_DIR ?= build
JOBS ?= $(shell nproc 2>/dev/null || echo 8)
PYTHON ?= python3

.PHONY: all build cmds test test-unit test-gpu coverage asan tsan asan-e2e tsan-e2e fuzz bench fmt assert-fmt vet lint check-yamls image image-offline shell clean

all: build

# Native daemon, C++ unit tests and the Python extension (in-tree).
build:
	cmake -S . -B $(BUILD_DIR) -G Ninja -DCMAKE_BUILD_TYPE=Release -DPython3_EXECUTABLE=$$(command -v $(PYTHON))
	cmake --build $(BUILD_DIR) -j $(JOBS)

cmds: build

# CPU test-suite (what CI runs): C++ unit tests + goldens + daemon + bench contract.
test: build
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-unit: build
	GFD_AMDSMI_LIBRARY=$(BUILD_DIR)/libfake_amdsmi.so ./$(BUILD_DIR)/gfd_unit_tests

# Real-hardware tests (MI355X): run on a GPU node.
test-gpu: build
	$(PYTHON) -m pytest tests -q -m gpu

# Sanitizer builds of the host code on the mock/synthetic backends (the
# reference runs `go test` without -race).
asan:
	cmake -S . -B build-asan -G Ninja -DCMAKE_BUILD_TYPE=Debug -DGFD_SANITIZE=address,undefined,float-cast-overflow -DGFD_BUILD_PYTHON=OFF
	cmake --build build-asan -j $(JOBS)
	ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1 GFD_AMDSMI_LIBRARY=build-asan/libfake_amdsmi.so ./build-asan/gfd_unit_tests
	for t in config pci values flags sysfs amdsmi; do ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1 \
	  ./build-asan/fuzz_replay_$$t tests/fuzz/corpus/$$t || exit 1; done

tsan:
	cmake -S . -B build-tsan -G Ninja -DCMAKE_BUILD_TYPE=Debug -DGFD_SANITIZE=thread -DGFD_BUILD_PYTHON=OFF
	cmake --build build-tsan -j $(JOBS)
	TSAN_OPTIONS=halt_on_error=1 GFD_AMDSMI_LIBRARY=build-tsan/libfake_amdsmi.so ./build-tsan/gfd_unit_tests

# The CPU test suite with the daemon binary and the fake amd-smi built under
# ASan/UBSan or TSan: every end-to-end, differential, soak and deployment test
# that runs the daemon runs the sanitized one.  Reports go to files, and any
# report fails the target (a test that only stops the daemon would not see
# it on stderr).  GFD_SANITIZED lifts the few timing bounds; TSan runs a
# shorter differential (it slows every fresh process ~10x).
SAN_LOGS ?= /tmp/gfd-san-logs
asan-e2e: asan
	rm -rf $(SAN_LOGS) && mkdir -p $(SAN_LOGS)
	ASAN_OPTIONS=detect_leaks=1:log_path=$(SAN_LOGS)/asan UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1:log_path=$(SAN_LOGS)/ubsan \
	  GFD_SANITIZED=1 GFD_BINARY=$(CURDIR)/build-asan/gpu-feature-discovery GFD_BUILD_DIR=$(CURDIR)/build-asan \
	  $(PYTHON) -m pytest tests -q -m "not gpu" -p no:cacheprovider
	@if ls $(SAN_LOGS)/* >/dev/null 2>&1; then cat $(SAN_LOGS)/*; exit 1; fi

tsan-e2e: tsan
	rm -rf $(SAN_LOGS) && mkdir -p $(SAN_LOGS)
	TSAN_OPTIONS=halt_on_error=1:log_path=$(SAN_LOGS)/tsan GFD_DIFF_SEQUENCES=40 \
	  GFD_SANITIZED=1 GFD_BINARY=$(CURDIR)/build-tsan/gpu-feature-discovery GFD_BUILD_DIR=$(CURDIR)/build-tsan \
	  $(PYTHON) -m pytest tests -q -m "not gpu" -p no:cacheprovider
	@if ls $(SAN_LOGS)/* >/dev/null 2>&1; then cat $(SAN_LOGS)/*; exit 1; fi

# libFuzzer + ASan/UBSan over the config reader, the PCI capability walkers
# and the value parsers (tests/fuzz/); FUZZ_SECONDS per target, new inputs
# kept in build-fuzz/corpus-<target>, seeds and regressions in tests/fuzz/corpus.
FUZZ_SECONDS ?= 60
FUZZ_CXX ?= $(shell command -v clang++ || echo /opt/rocm/lib/llvm/bin/clang++)
fuzz:
	cmake -S . -B build-fuzz -G Ninja -DCMAKE_BUILD_TYPE=Debug -DCMAKE_CXX_COMPILER=$(FUZZ_CXX) \
	  -DGFD_SANITIZE=address,undefined -DGFD_FUZZ=ON -DGFD_BUILD_PYTHON=OFF -DGFD_BUILD_TESTS=OFF
	cmake --build build-fuzz -j $(JOBS)
	for t in config pci values flags sysfs amdsmi; do mkdir -p build-fuzz/corpus-$$t && \
	  UBSAN_OPTIONS=halt_on_error=1 ./build-fuzz/fuzz_$$t -max_total_time=$(FUZZ_SECONDS) -timeout=10 \
	    -rss_limit_mb=2048 $$([ -f tests/fuzz/$$t.dict ] && echo -dict=tests/fuzz/$$t.dict) \
	    build-fuzz/corpus-$$t tests/fuzz/corpus/$$t || exit 1; done

coverage:
	cmake -S . -B build-cov -G Ninja -DCMAKE_BUILD_TYPE=Debug -DGFD_BUILD_PYTHON=OFF \
	  -DCMAKE_CXX_FLAGS="--coverage" -DCMAKE_EXE_LINKER_FLAGS="--coverage"
	cmake --build build-cov -j $(JOBS)
	find build-cov -name '*.gcda' -delete
	./build-cov/gfd_unit_tests > /dev/null
	GFD_AMDSMI_LIBRARY=build-cov/libfake_amdsmi.so ./build-cov/gfd_unit_tests > /dev/null
	# The daemon binary under the Python end-to-end tests and the fuzz-corpus
	# replays add their own counts.
	GFD_BINARY=$(CURDIR)/build-cov/gpu-feature-discovery GFD_BUILD_DIR=$(CURDIR)/build-cov $(PYTHON) -m pytest tests -q -m "not gpu" -p no:cacheprovider
	@for f in src/*/*.cpp; do gcov -n -o build-cov/CMakeFiles/gfdcore.dir/$$f.o $$f 2>/dev/null | \
	  grep -A1 "^File '.*$$f'" | tail -1 | sed "s|Lines executed:|$$f |"; done | \
	  awk '{split($$2, p, "%"); n = $$4; hit += p[1] * n / 100; tot += n; print} \
	       END {printf "TOTAL %.1f%% of %d lines\n", 100 * hit / tot, tot}'

bench: build
	$(PYTHON) bench.py

fmt:
	find src tests/unit python -name '*.cpp' -o -name '*.h' | xargs clang-format -i

assert-fmt:
	find src tests/unit python -name '*.cpp' -o -name '*.h' | xargs clang-format --dry-run --Werror

# Static checks of the C++ (reference analogue: `go vet`, Makefile:102-103):
# the whole tree built by clang with extra diagnostics, every warning an error.
VET_FLAGS = -Werror -Wshadow -Wnon-virtual-dtor -Wnull-dereference -Wformat=2 -Wdeprecated -Wcomma -Wloop-analysis \
  -Wunused-member-function -Wconditional-uninitialized -Wextra-semi -Wunreachable-code -Wimplicit-fallthrough
vet:
	cmake -S . -B build-vet -G Ninja -DCMAKE_BUILD_TYPE=Release -DCMAKE_CXX_COMPILER=$(FUZZ_CXX) \
	  -DGFD_BUILD_PYTHON=OFF -DCMAKE_CXX_FLAGS="$(VET_FLAGS)"
	cmake --build build-vet -j $(JOBS)

LINT_PY = gpu_feature_discovery_amd tests tools bench.py __graft_entry__.py
lint:
	@if $(PYTHON) -c "import pyflakes" 2>/dev/null; then $(PYTHON) -m pyflakes $(LINT_PY); \
	else echo "pyflakes not installed (make docker-lint has it): byte-compiling only"; \
	  $(PYTHON) -m compileall -q $(LINT_PY) > /dev/null; fi

check-yamls:
	$(PYTHON) -m pytest tests/test_deployments.py -q

image:
	$(MAKE) -C deployments/container image VERSION=$(VERSION) IMAGE_NAME=$(IMAGE_NAME)

# The same Dockerfile built without docker (no image builder on the GPU pool):
# its build stage run in a copy of the build context, the runtime stage
# assembled from the result and its entrypoint run (tools/image_build.py).
image-offline:
	$(PYTHON) tools/image_build.py

# Any target inside the development image (reference analogue: the
# docker-% targets, Makefile:119-150): `make docker-test`, `make docker-asan`...
DOCKER ?= docker
BUILDIMAGE ?= $(IMAGE_NAME)-devel:$(VERSION)

.build-image: docker/Dockerfile.devel
	$(DOCKER) build --build-arg ROCM_VERSION=$(basename $(ROCM_VERSION)) \
	  --build-arg UBUNTU_VERSION=$(UBUNTU_VERSION) --tag $(BUILDIMAGE) -f docker/Dockerfile.devel docker

docker-%: .build-image
	$(DOCKER) run --rm -v $(CURDIR):/work -w /work --user $$(id -u):$$(id -g) -e HOME=/tmp \
	  $(BUILDIMAGE) make $*

shell: .build-image
	$(DOCKER) run --rm -ti -v $(CURDIR):/work -w /work --user $$(id -u):$$(id -g) -e HOME=/tmp $(BUILDIMAGE)

clean:
	rm -rf $(BUILD_DIR) build-asan build-tsan build-cov build-vet gpu_feature_discovery_amd/_gfd*.so
