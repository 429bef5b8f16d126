# Top-level build: the product library (libtips_hip.so, gfx950 only: exactly the C-ABI of
# include/tips_hip.h), the development library (tools/lib/libtips_hip_dev.so: the same runtime plus
# include/tips_hip_dev.h's simulators, self-tests and tuning sweeps, -DTIPS_DEV) and the oracle checkers.
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
LIB      := tips_amd/lib/libtips_hip.so
SRCS     := tips_amd/csrc/kernels.hip tips_amd/csrc/runtime.cc tips_amd/csrc/rt_common.cc tips_amd/csrc/plan.cc tips_amd/csrc/schedules.cc \
            tips_amd/csrc/fusion.cc tips_amd/csrc/host_staging.cc tips_amd/csrc/control.cc tips_amd/csrc/negotiate.cc tips_amd/csrc/peer.cc \
            tips_amd/csrc/bootstrap.cc
HDRS     := tips_amd/csrc/kernels.h tips_amd/csrc/rt.h tips_amd/csrc/net.h tips_amd/csrc/plan.h include/tips_hip.h \
            include/tips_hip_dev.h
DEVLIB   := tools/lib/libtips_hip_dev.so
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fno-gpu-flush-denormals-to-zero -Wall -Wno-unused-result -fvisibility=hidden

CRASH    := tools/lib/libcrashline.so

REPRO    := tools/_bin/graph_repro tools/_bin/graph_probe tools/_bin/op_body tools/_bin/op_host tools/_bin/op_host_check \
            tools/_bin/capture_race tools/_bin/capture_race_hip

FAST     := tips_amd/_fast$(shell python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
TORCH    := $(shell python3 -c "import os, torch; print(os.path.dirname(torch.__file__))" 2>/dev/null)
PYINC    := $(shell python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")

all: $(LIB) $(DEVLIB) $(FAST) $(CRASH) $(REPRO) oracle tsan tools/cpu_sum_bench

# the Python mirror's list helper (tips_amd._fast: tensor pointers / counts in C++), torch headers
$(FAST): tips_amd/csrc/pyfast.cc
	g++ -O2 -std=c++17 -shared -fPIC -Wall -D_GLIBCXX_USE_CXX11_ABI=1 -I$(PYINC) -I$(TORCH)/include \
	  -I$(TORCH)/include/torch/csrc/api/include -o $@ $< -L$(TORCH)/lib -ltorch_python -ltorch -lc10 \
	  -Wl,-rpath,$(TORCH)/lib

# bench.py's last-words hook (not part of the product library)
$(CRASH): tools/crash_line.c
	@mkdir -p tools/lib
	gcc -O2 -fPIC -shared -Wall -Wextra -std=c11 -D_POSIX_C_SOURCE=200809L -o $@ $<

OBJS     := $(patsubst tips_amd/csrc/%,build/obj/%.o,$(SRCS))

# one object per source (parallel, incremental); every object depends on every internal header
build/obj/%.o: tips_amd/csrc/% $(HDRS)
	@mkdir -p build/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# -Bsymbolic: each library calls its own entry points (the development library is loaded beside the
# product one in test processes, RTLD_LOCAL: its internal calls must not bind to the product's copies)
$(LIB): $(OBJS)
	@mkdir -p tips_amd/lib
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-Bsymbolic -o $@ $(OBJS) -lrccl

DEV_OBJS := $(patsubst tips_amd/csrc/%,build/dev/%.o,$(SRCS))

build/dev/%.o: tips_amd/csrc/% $(HDRS)
	@mkdir -p build/dev
	$(HIPCC) $(HIPFLAGS) -DTIPS_DEV -c -o $@ $<

$(DEVLIB): $(DEV_OBJS)
	@mkdir -p tools/lib
	$(HIPCC) $(HIPFLAGS) -shared -Wl,-Bsymbolic -o $@ $(DEV_OBJS) -lrccl

# replayed-plan checks through the C-ABI on /opt/rocm's runtime (tests/test_gpu_graphs.py)
tools/_bin/graph_repro: tools/graph_repro.cc $(LIB) include/tips_hip.h
	@mkdir -p tools/_bin
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Iinclude -o $@ $< -Ltips_amd/lib -ltips_hip -Wl,-rpath,'$$ORIGIN/../../tips_amd/lib'

# the op-body pattern through the C-ABI in a plain-C host (tests/test_gpu_op_body.py): checked
# against the oracle's fold, so it links oracle/build/liboracle.so (test infrastructure only)
tools/_bin/op_body: tests/c/op_body.c $(LIB) include/tips_hip.h oracle/build/liboracle.so
	@mkdir -p tools/_bin
	gcc -O2 -std=gnu11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle -o $@ $< \
	  -Ltips_amd/lib -ltips_hip -Loracle/build -loracle -L/opt/rocm/lib -lamdhip64 -lpthread \
	  -Wl,-rpath,'$$ORIGIN/../../tips_amd/lib' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -Wl,-rpath,/opt/rocm/lib

# direct tips_allreduce captures on one thread while other threads make HIP calls (tests/test_gpu_op_body.py)
tools/_bin/capture_race: tests/c/capture_race.c $(LIB) include/tips_hip.h oracle/build/liboracle.so
	@mkdir -p tools/_bin
	gcc -O2 -std=gnu11 -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle -o $@ $< \
	  -Ltips_amd/lib -ltips_hip -Loracle/build -loracle -L/opt/rocm/lib -lamdhip64 -lpthread \
	  -Wl,-rpath,'$$ORIGIN/../../tips_amd/lib' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -Wl,-rpath,/opt/rocm/lib

# the same capture pattern on the HIP runtime alone, no RCCL and no library (diagnostic)
tools/_bin/capture_race_hip: tools/capture_race_hip.cc
	@mkdir -p tools/_bin
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -o $@ $< -lpthread

# what the HIP calls of a named-request enqueue cost (diagnostic, tools/enqueue_probe.cc)
tools/_bin/enqueue_probe: tools/enqueue_probe.cc
	@mkdir -p tools/_bin
	$(HIPCC) -O2 -std=c++17 --offload-arch=$(ARCH) -o $@ $< -lpthread

# config 5 as 214 named host requests from TF-style executor threads (tools/op_host.c): bench.py's
# leg links the product library only; the -m gpu test's build also checks against the oracle's fold
tools/_bin/op_host: tools/op_host.c $(LIB) include/tips_hip.h
	@mkdir -p tools/_bin
	gcc -O2 -std=gnu11 -Wall -Iinclude -o $@ $< -Ltips_amd/lib -ltips_hip -lpthread -Wl,-rpath,'$$ORIGIN/../../tips_amd/lib'

tools/_bin/op_host_check: tools/op_host.c $(LIB) include/tips_hip.h oracle/build/liboracle.so
	@mkdir -p tools/_bin
	gcc -O2 -std=gnu11 -Wall -DOP_HOST_ORACLE -Iinclude -Ioracle -o $@ $< -Ltips_amd/lib -ltips_hip -Loracle/build -loracle \
	  -lpthread -Wl,-rpath,'$$ORIGIN/../../tips_amd/lib' -Wl,-rpath,'$$ORIGIN/../../oracle/build'

oracle/build/liboracle.so: oracle/oracle.c oracle/oracle.h
	$(MAKE) -C oracle build/liboracle.so

# ThreadSanitizer build of the same sources (host code only: -fsanitize=thread after -Xarch_host;
# device code unchanged) and its CPU driver - tests/test_tsan.py (the negotiation with threads and
# callbacks, the host copy pool); tools/_bin/op_body_tsan runs the op-body test on the GPU box
TSAN_OBJS := $(patsubst tips_amd/csrc/%,build/tsan/%.o,$(SRCS))
TSAN_LIB  := tools/lib/libtips_hip_tsan.so
CLANG     := /opt/rocm/lib/llvm/bin/clang

build/tsan/%.o: tips_amd/csrc/% $(HDRS)
	@mkdir -p build/tsan
	$(HIPCC) --offload-arch=$(ARCH) -O1 -g -std=c++17 -fPIC -fno-gpu-flush-denormals-to-zero -fvisibility=hidden \
	  -DTIPS_DEV -Xarch_host -fsanitize=thread -c -o $@ $<

$(TSAN_LIB): $(TSAN_OBJS)
	@mkdir -p tools/lib
	$(HIPCC) --offload-arch=$(ARCH) -shared -o $@ $(TSAN_OBJS) -lrccl

tools/_bin/tsan_selftest: tools/tsan_selftest.c $(TSAN_LIB) include/tips_hip.h
	@mkdir -p tools/_bin
	$(CLANG) -O1 -g -fsanitize=thread -Iinclude -o $@ $< -Ltools/lib -ltips_hip_tsan -Wl,-rpath,'$$ORIGIN/../lib'

tools/_bin/op_body_tsan: tests/c/op_body.c $(TSAN_LIB) include/tips_hip.h oracle/build/liboracle.so
	@mkdir -p tools/_bin
	$(CLANG) -O1 -g -fsanitize=thread -std=gnu11 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -Ioracle -o $@ $< \
	  -Ltools/lib -ltips_hip_tsan -Loracle/build -loracle -L/opt/rocm/lib -lamdhip64 -lpthread \
	  -Wl,-rpath,'$$ORIGIN/../lib' -Wl,-rpath,'$$ORIGIN/../../oracle/build' -Wl,-rpath,/opt/rocm/lib

tsan: tools/_bin/tsan_selftest tools/_bin/op_body_tsan

tools/_bin/graph_probe: tools/graph_probe.cc
	@mkdir -p tools/_bin
	$(HIPCC) --offload-arch=$(ARCH) -O2 -o $@ $< -lrccl

repro: $(REPRO)

oracle:
	$(MAKE) -C oracle

tools: tools/sum_sweep tools/cpu_sum_bench tools/peer_mem_probe tools/ipc_probe

tools/peer_mem_probe: tools/peer_mem_probe.cc $(DEVLIB)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Iinclude -o $@ $< -Ltools/lib -ltips_hip_dev -Wl,-rpath,'$$ORIGIN/lib'

tools/ipc_probe: tools/ipc_probe.cc
	$(HIPCC) --offload-arch=$(ARCH) -O2 -o $@ $<

tools/cpu_sum_bench: tools/cpu_sum_bench.c
	gcc -O3 -fopenmp -o $@ $<

tools/sum_sweep: tools/sum_sweep.cc $(DEVLIB)
	$(HIPCC) -O2 -std=c++17 -o $@ $< -Iinclude -Ltools/lib -ltips_hip_dev -Wl,-rpath,'$$ORIGIN/lib'

clean:
	rm -rf build/obj build/dev
	rm -f $(LIB) $(DEVLIB) $(REPRO) tools/sum_sweep tools/cpu_sum_bench tools/peer_mem_probe tools/ipc_probe
	$(MAKE) -C oracle clean

.PHONY: all oracle tools repro clean tsan
