# Build of the MI355X engine (gfx950 only) and of its test infrastructure.
#   make lib      narwhal_amd/lib/libnwv.so   (product: HIP kernels + C ABI, include/nwv.h)
#   make oracle   oracle/build/libnwv_oracle.so (test infrastructure: CPU restatement)
#   make hostemu  tests/_build/libhostemu.so    (test infrastructure: device math on the host)
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
BLS_SRC := narwhal_amd/csrc/nwv_bls.hip narwhal_amd/csrc/bls381.h narwhal_amd/csrc/bls_verify.h narwhal_amd/csrc/bls_group.h \
	narwhal_amd/csrc/bls381_consts.h narwhal_amd/csrc/bls381_iso.h narwhal_amd/csrc/bls_wave.h \
	narwhal_amd/csrc/bls_wave_prog.h narwhal_amd/csrc/bls_shard.h include/nwv_bls.h
CSRC := $(filter-out $(BLS_SRC),$(wildcard narwhal_amd/csrc/*.h narwhal_amd/csrc/*.hip narwhal_amd/csrc/*.cpp)) \
	include/nwv.h include/nwv_types.h include/nwv_service.h

all: lib oracle hostemu tools

lib: narwhal_amd/lib/libnwv.so
# nwv_types.cpp is plain host C++ (no kernels): built by g++ on its own, because mixing `-x c++`
# into the hipcc line makes hipcc drop --offload-arch (the code object silently falls back to gfx906)
narwhal_amd/lib/nwv_types.o: narwhal_amd/csrc/nwv_types.cpp include/nwv.h include/nwv_types.h include/nwv_bls.h
	@mkdir -p narwhal_amd/lib
	g++ -O2 -std=c++17 -fPIC -Wall -c -o $@ $<
narwhal_amd/lib/nwv_service.o: narwhal_amd/csrc/nwv_service.cpp include/nwv.h include/nwv_types.h include/nwv_service.h
	@mkdir -p narwhal_amd/lib
	g++ -O2 -std=c++17 -fPIC -Wall -c -o $@ $<
# the BLS12-381 engine is its own translation unit (compiled in parallel with the Ed25519 one)
narwhal_amd/lib/nwv_bls.o: $(BLS_SRC) include/nwv.h
	@mkdir -p narwhal_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -c -o $@ narwhal_amd/csrc/nwv_bls.hip
narwhal_amd/lib/nwv_host.o: $(CSRC)
	@mkdir -p narwhal_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Wall -c -o $@ narwhal_amd/csrc/nwv_host.hip
narwhal_amd/lib/libnwv.so: narwhal_amd/lib/nwv_host.o narwhal_amd/lib/nwv_bls.o narwhal_amd/lib/nwv_types.o \
		narwhal_amd/lib/nwv_service.o
	@mkdir -p narwhal_amd/lib
	$(HIPCC) --offload-arch=$(ARCH) -fPIC -shared -o $@ narwhal_amd/lib/nwv_host.o narwhal_amd/lib/nwv_bls.o \
		narwhal_amd/lib/nwv_types.o narwhal_amd/lib/nwv_service.o -lpthread

oracle:
	$(MAKE) -C oracle

hostemu: tests/_build/libhostemu.so tests/_build/libsvcstub.so tests/_build/libblsemu.so tests/_build/libblsshard.so
# the BLS and Ed25519 calls' split over a multi-device context (bls_shard.h, shard.h) with stub per-device work
tests/_build/libblsshard.so: tests/hostemu/bls_shard_stub.cpp narwhal_amd/csrc/bls_shard.h narwhal_amd/csrc/shard.h
	@mkdir -p tests/_build
	g++ -O1 -g -std=c++17 -fPIC -shared -pthread -o $@ tests/hostemu/bls_shard_stub.cpp
# the gfx950 BLS12-381 code compiled for the host (tests/test_bls_hostemu.py)
tests/_build/libblsemu.so: tests/hostemu/bls_hostemu.cpp $(BLS_SRC)
	@mkdir -p tests/_build
	$(HIPCC) -std=c++17 -O2 --offload-host-only -x hip -fPIC -shared -o $@ tests/hostemu/bls_hostemu.cpp
# the same build under AddressSanitizer + UndefinedBehaviorSanitizer (host code only):
#   make blsemu-asan && tools/run_blsemu_asan.sh
tests/_build/libblsemu_asan.so: tests/hostemu/bls_hostemu.cpp $(BLS_SRC)
	@mkdir -p tests/_build
	$(HIPCC) -std=c++17 -O1 -g --offload-host-only -x hip -fPIC -shared -fno-omit-frame-pointer \
		-fno-gpu-sanitize -fsanitize=address,undefined -fno-sanitize-recover=all -shared-libsan \
		-o $@ tests/hostemu/bls_hostemu.cpp
blsemu-asan: tests/_build/libblsemu_asan.so
# the batching service's host logic over a stubbed engine (tests/test_service_host.py)
tests/_build/libsvcstub.so: tests/hostemu/service_stub.cpp narwhal_amd/csrc/nwv_service.cpp include/nwv_service.h
	@mkdir -p tests/_build
	g++ -O1 -g -std=c++17 -fPIC -shared -pthread -o $@ tests/hostemu/service_stub.cpp narwhal_amd/csrc/nwv_service.cpp
tests/_build/libhostemu.so: tests/hostemu/hostemu.cpp $(CSRC)
	@mkdir -p tests/_build
	$(HIPCC) -std=c++17 -O1 --offload-host-only -x hip -DNWV_BOUNDS_CHECK -fPIC -shared -o $@ tests/hostemu/hostemu.cpp

tools: tools/ubench_valu tools/ubench_field tools/ubench_wave tools/ubench_row tools/ubench_prep tools/libsvcbench.so
# native drivers of the C5 service leg (bench tooling): the service and the Core drain timed from C++ threads
tools/libsvcbench.so: tools/svcbench.cpp narwhal_amd/lib/libnwv.so include/nwv.h include/nwv_types.h include/nwv_service.h
	g++ -O2 -std=c++17 -fPIC -shared -pthread -Wall -o $@ $< -Lnarwhal_amd/lib -lnwv -Wl,-rpath,'$$ORIGIN/../narwhal_amd/lib'
tools/ubench_valu: tools/ubench_valu.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -o $@ $<
tools/ubench_field: tools/ubench_field.hip narwhal_amd/csrc/fe25519.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
tools/ubench_wave: tools/ubench_wave.hip $(BLS_SRC)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -o $@ $<
tools/ubench_row: tools/ubench_row.hip narwhal_amd/csrc/fe_row.h narwhal_amd/csrc/msm.h
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Wno-unused-value -o $@ $<
tools/ubench_prep: tools/ubench_prep.hip $(CSRC)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Wno-unused-value -o $@ $<

clean:
	rm -rf narwhal_amd/lib tests/_build
	$(MAKE) -C oracle clean

.PHONY: blsemu-asan all lib oracle hostemu tools clean
