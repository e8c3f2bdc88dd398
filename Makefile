# Build of the product library (HIP, gfx950) and the CPU oracle (test infrastructure).
#   make            -> orb_slam3_comments_ghr_amd/liborbslam3_amd.so + oracle/liboracle.so
HIPCC ?= hipcc
ARCH ?= gfx950
PKG = orb_slam3_comments_ghr_amd
CSRC = $(PKG)/csrc
LIB = $(PKG)/liborbslam3_amd.so
OBJDIR = build/obj
HIPFLAGS = --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-function
# bit-exact float geometry in the matcher and BowVector sums: no FMA contraction in those units
EXACT = -ffp-contract=off
# make POSE_PROF=1: phase cycle counters in k_pose_opt (tools/pose_prof.py)
ifdef POSE_PROF
HIPFLAGS += -DOSG_POSE_PROF
endif
# make SR_PROF=1: k_schur_rows_c's per-workgroup timeline (tools/sr_prof.py)
ifdef SR_PROF
HIPFLAGS += -DOSG_SR_PROF
endif
HDRS = include/osg.h include/osg_ba.h $(CSRC)/osg_internal.h

OBJS = $(OBJDIR)/runtime.o $(OBJDIR)/hamming.o $(OBJDIR)/hamming_mfma.o $(OBJDIR)/match.o $(OBJDIR)/pose.o $(OBJDIR)/ba.o $(OBJDIR)/dbow.o $(OBJDIR)/fuse.o $(OBJDIR)/triang.o $(OBJDIR)/desc.o $(OBJDIR)/sim3.o $(OBJDIR)/init.o $(OBJDIR)/stereo.o $(OBJDIR)/orb.o $(OBJDIR)/fast.o $(OBJDIR)/pyramid.o

WALL_BENCH = tools/adapter_wall_bench

all: $(LIB) oracle $(WALL_BENCH)

$(OBJDIR):
	mkdir -p $(OBJDIR)

$(OBJDIR)/runtime.o: $(CSRC)/runtime.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(OBJDIR)/hamming.o: $(CSRC)/hamming.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@
$(OBJDIR)/hamming_mfma.o: $(CSRC)/hamming_mfma.hip $(HDRS) | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(OBJDIR)/match.o: $(CSRC)/match.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@
$(OBJDIR)/pose.o: $(CSRC)/pose.hip $(HDRS) $(CSRC)/ba_common.h $(CSRC)/exact_math.h $(CSRC)/glibc_math.h $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@
$(OBJDIR)/ba.o: $(CSRC)/ba.hip $(HDRS) $(CSRC)/ba_common.h $(CSRC)/exact_math.h $(CSRC)/glibc_math.h $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
$(OBJDIR)/dbow.o: $(CSRC)/dbow.hip $(HDRS) include/osg_dbow.h $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/fuse.o: $(CSRC)/fuse.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/triang.o: $(CSRC)/triang.hip $(HDRS) $(CSRC)/match_common.h $(CSRC)/kb8_epipolar.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/desc.o: $(CSRC)/desc.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/sim3.o: $(CSRC)/sim3.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/init.o: $(CSRC)/init.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/stereo.o: $(CSRC)/stereo.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/orb.o: $(CSRC)/orb.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/fast.o: $(CSRC)/fast.hip $(HDRS) $(CSRC)/match_common.h $(CSRC)/octree.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(OBJDIR)/pyramid.o: $(CSRC)/pyramid.hip $(HDRS) $(CSRC)/match_common.h | $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) $(EXACT) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# the C++ adapter wall-rate bench (bench.py's wall_cpp_adapter_frames_per_s): host code over the
# library and the HIP runtime (device-resident pyramid levels for the stereo workload)
$(WALL_BENCH): tools/adapter_wall_bench.cpp adapters/orbslam3/osg_orbslam3.h tests/adapter/driver_common.h tests/adapter/mock_orbslam3.h include/osg.h include/osg_ba.h include/osg_dbow.h $(LIB)
	g++ -std=c++17 -O2 -Wall -Werror -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude $< -o $@ -L$(PKG) -lorbslam3_amd -L/opt/rocm/lib -lamdhip64 '-Wl,-rpath,$$ORIGIN/../$(PKG)' -Wl,-rpath,/opt/rocm/lib -pthread
