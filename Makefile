# In-tree build: the .so files travel to the GPU box with the gpurun snapshot.
#   build/librtmi355x.so   HIP kernels + C ABI (include/rt_mi355x.h)   <- the product
#   build/librthost.so     C++ scene builder + output stage (include/rt_host.h)
#   build/rt_render_cli    main.rs-equivalent host program (preset -> PPM)
#   build/librtgather.so   RCCL framebuffer gather for one process per GPU (include/rt_gather.h)
#   oracle/_build/*.so     CPU restatement (test infrastructure only)
PKG      := surely-raytracing_amd
CSRC     := $(PKG)/csrc
BUILD    := build
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# device path is f64; contraction off, fma written explicitly (deterministic bits)
HIPFLAGS := --offload-arch=$(ARCH) -Iinclude -I$(BUILD) -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function
CXXFLAGS := -O2 -std=c++17 -fPIC -Wall -Wextra
CFLAGS_O := -std=c11 -O2 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function

HOST_SRC := $(CSRC)/host/scene.cpp $(CSRC)/host/presets.cpp $(CSRC)/host/capi.cpp
DEV_SRC  := $(CSRC)/rt_device.hip $(CSRC)/rt_flatten.cpp $(CSRC)/rt_obvh.cpp $(CSRC)/rt_jit.cpp
DEV_HDR  := $(CSRC)/rt_kernel.h $(CSRC)/rt_rng.h $(CSRC)/rt_layout.h $(CSRC)/rt_flatten.hpp $(CSRC)/rt_jit.hpp include/rt_mi355x.h $(BUILD)/rt_jit_sources.inc
JIT_HDR  := $(CSRC)/rt_kernel.h $(CSRC)/rt_layout.h include/rt_mi355x.h $(CSRC)/rt_rng.h

.PHONY: all device host oracle cli gather clean
all: device host oracle cli gather

device: $(BUILD)/librtmi355x.so
host: $(BUILD)/librthost.so
cli: $(BUILD)/rt_render_cli
gather: $(BUILD)/librtgather.so
oracle: oracle/_build/liboracle_f32.so oracle/_build/liboracle_f64.so oracle/_build/liboracle_f64fma.so

# device headers embedded for the scene-specialised kernels compiled at run time (rt_jit.cpp)
$(BUILD)/rt_jit_sources.inc: $(JIT_HDR) $(CSRC)/embed_sources.py
	@mkdir -p $(BUILD)
	python3 $(CSRC)/embed_sources.py $@ $(JIT_HDR)

# one object per source, so an edit of the host-side generator or flattener does not recompile
# the kernels (rt_device.hip: every ahead-of-time template instance, ~3 minutes)
OBJ      := $(BUILD)/obj
DEV_OBJ  := $(OBJ)/rt_device.o $(OBJ)/rt_flatten.o $(OBJ)/rt_obvh.o $(OBJ)/rt_jit.o
$(OBJ)/rt_device.o: $(CSRC)/rt_device.hip $(DEV_HDR)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(OBJ)/%.o: $(CSRC)/%.cpp $(DEV_HDR)
	@mkdir -p $(OBJ)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/librtmi355x.so: $(DEV_OBJ)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -shared $(DEV_OBJ) -o $@ -lhiprtc

$(BUILD)/librtgather.so: $(CSRC)/rt_gather.hip include/rt_gather.h include/rt_mi355x.h
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -shared $(CSRC)/rt_gather.hip -o $@ -lrccl

$(BUILD)/librthost.so: $(HOST_SRC) $(CSRC)/host/scene.hpp include/rt_host.h include/rt_mi355x.h
	@mkdir -p $(BUILD)
	g++ $(CXXFLAGS) -shared $(HOST_SRC) -o $@

$(BUILD)/rt_render_cli: $(CSRC)/host/rt_render_cli.cpp $(BUILD)/librthost.so $(BUILD)/librtmi355x.so
	g++ $(CXXFLAGS) $< -o $@ -L$(BUILD) -lrthost -lrtmi355x -Wl,-rpath,'$$ORIGIN'

oracle/_build/liboracle_f32.so: oracle/rt_oracle.c include/rt_mi355x.h
	@mkdir -p oracle/_build
	gcc $(CFLAGS_O) -DORACLE_F64=0 -shared $< -o $@ -lpthread -lm

oracle/_build/liboracle_f64.so: oracle/rt_oracle.c include/rt_mi355x.h
	@mkdir -p oracle/_build
	gcc $(CFLAGS_O) -DORACLE_F64=1 -shared $< -o $@ -lpthread -lm

# perturbation study (tools/flip_study.py): the f64 oracle with fused dot products
oracle/_build/liboracle_f64fma.so: oracle/rt_oracle.c include/rt_mi355x.h
	@mkdir -p oracle/_build
	gcc $(CFLAGS_O) -DORACLE_F64=1 -DORACLE_FMA_DOT=1 -shared $< -o $@ -lpthread -lm

clean:
	rm -rf $(BUILD) oracle/_build

# performance variants for A/B measurement (tools_gpu/ab_variants.py); not shipped
VARIANTS := $(BUILD)/variants
variants: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(VARIANTS)
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_TRAV2 -shared $(DEV_SRC) -o $(VARIANTS)/librtmi355x_abl_trav2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_LPDF2 -shared $(DEV_SRC) -o $(VARIANTS)/librtmi355x_abl_lpdf2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_FRESH2 -shared $(DEV_SRC) -o $(VARIANTS)/librtmi355x_abl_fresh2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_HIT2 -shared $(DEV_SRC) -o $(VARIANTS)/librtmi355x_abl_hit2.so -lhiprtc

# occupancy variants of the BVH kernels; A/B with
# VARDIR=build/variants_occ python tools_gpu/ab_variants.py W SPP ROUNDS SCENE
variants-occ: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_occ
	$(HIPCC) $(HIPFLAGS) -DRT_MIN_WAVES_BVH=2 -DRT_BLOCK_BVH=512 -shared $(DEV_SRC) -o $(BUILD)/variants_occ/librtmi355x_bvh2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_MIN_WAVES_BVH=4 -shared $(DEV_SRC) -o $(BUILD)/variants_occ/librtmi355x_bvh4.so -lhiprtc

# section-cycle profiling build (tools_gpu/prof_sections.py); not shipped
prof: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/prof
	$(HIPCC) $(HIPFLAGS) -DRT_PROF -shared $(DEV_SRC) -o $(BUILD)/prof/librtmi355x.so -lhiprtc

# occupancy variants of the non-BVH kernels (the scene-specialised C2/C3 kernels inherit
# RT_MIN_WAVES through rt_jit.cpp); A/B with
# VARDIR=build/variants_jocc python tools_gpu/ab_variants.py W SPP ROUNDS SCENE
variants-jocc: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_jocc
	$(HIPCC) $(HIPFLAGS) -DRT_MIN_WAVES=3 -shared $(DEV_SRC) -o $(BUILD)/variants_jocc/librtmi355x_w3.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_MIN_WAVES=5 -shared $(DEV_SRC) -o $(BUILD)/variants_jocc/librtmi355x_w5.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_MIN_WAVES=6 -shared $(DEV_SRC) -o $(BUILD)/variants_jocc/librtmi355x_w6.so -lhiprtc

# C4 ablations: every BVH leaf tested twice (variants-c4), the top-level / in-instance walk run
# twice (variants-c4-walks)
# (its cost); A/B with VARDIR=build/variants_c4 python tools_gpu/ab_variants.py 800 400 3 final_scene
variants-c4: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_c4
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_LEAF2 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_leaf2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_NOISE2 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_noise2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_FRESH2 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_fresh2.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_HIT2 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_hit2.so -lhiprtc

# upper bound of resumable top-level walks (wrong images): walks cut after K box steps
variants-c4-budget: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_c4b
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_BUDGET=6 -shared $(DEV_SRC) -o $(BUILD)/variants_c4b/librtmi355x_b06.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_BUDGET=10 -shared $(DEV_SRC) -o $(BUILD)/variants_c4b/librtmi355x_b10.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_BUDGET=14 -shared $(DEV_SRC) -o $(BUILD)/variants_c4b/librtmi355x_b14.so -lhiprtc

variants-c4-walks: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_c4
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_TWICE_BVH=1 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_twice1.so -lhiprtc
	$(HIPCC) $(HIPFLAGS) -DRT_ABL_TWICE_BVH=2 -shared $(DEV_SRC) -o $(BUILD)/variants_c4/librtmi355x_twice2.so -lhiprtc

# cost probe of reference-order arithmetic (unfused products, IEEE division/sqrt); not shipped
variants-exact: $(DEV_SRC) $(DEV_HDR)
	@mkdir -p $(BUILD)/variants_exact
	$(HIPCC) $(HIPFLAGS) -DRT_EXACT_PROBE -shared $(DEV_SRC) -o $(BUILD)/variants_exact/librtmi355x_exact.so -lhiprtc
