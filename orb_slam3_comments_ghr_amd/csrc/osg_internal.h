// osg_internal.h — shared host/device internals of liborbslam3_amd (not part of the ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/osg.h"
#include "../../include/osg_ba.h"

// Scratch slots: each entry point owns a few named device buffers that grow on demand and are
// reused across calls (no hipMalloc on the steady-state path).
enum osg_slot {
    SLOT_Q = 0, SLOT_T, SLOT_OUT, SLOT_PART, SLOT_TMP0, SLOT_TMP1, SLOT_TMP2, SLOT_TMP3,
    SLOT_TMP4, SLOT_TMP5, SLOT_TMP6, SLOT_TMP7, SLOT_TMP8, SLOT_TMP9, SLOT_TMP10, SLOT_TMP11,
    SLOT_BA0, SLOT_BA1, SLOT_BA2, SLOT_BA3, SLOT_BA4, SLOT_BA5, SLOT_BA6, SLOT_BA7,
    SLOT_BA8, SLOT_BA9, SLOT_BA10, SLOT_BA11, SLOT_BA12, SLOT_BA13, SLOT_BA14, SLOT_BA15,
    SLOT_PINNED0, SLOT_COUNT
};

// Counters for in-launch last-arriver merges: zero at allocation, each launch leaves them zero.
#define OSG_N_COUNTERS 65536

struct osg_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    void *buf[SLOT_COUNT] = {};
    size_t cap[SLOT_COUNT] = {};
    void *host_pinned = nullptr;
    size_t host_pinned_cap = 0;
    uint32_t *counters = nullptr;
    int num_cus = 256;
    int lds_per_block = 65536;
    int32_t match_stats[4] = {};  // last matcher call: candidates, Jacobi rounds, serial redo, nmatches
    double last_kernel_ms = 0;    // last k_match / k_pose_opt launch time (HIP events)
    hipEvent_t ev[2] = {};        // timing events (osg_ctx_events)
    hipEvent_t ev_done = nullptr; // completion marker of osg_wait (no timing)
    unsigned long long *lb_flags = nullptr;  // k_grid_prepass's per-workgroup counts (epoch-tagged)
    size_t lb_cap = 0;
    uint32_t lb_epoch = 0;
    std::shared_ptr<void> lba_cache;  // host structures of the last LBA batch, reused (ba.hip)
    std::shared_ptr<void> match_cache;  // the matchers' per-problem host arrays, reused (match.hip)
    bool lba_ktime = false;           // osg_lba_kernel_times: per-kernel HIP-event timing of LBA steps
    double lba_kms[OSG_LBA_NK] = {};
    int64_t lba_kn[OSG_LBA_NK] = {};
    std::string last_error;
};

int osg_set_error(osg_ctx *ctx, int code, const char *fmt, ...);
// the context's two timing events, created on first use (nullptr on failure)
hipEvent_t *osg_ctx_events(osg_ctx *ctx);
// device buffer of at least `bytes` for `slot` (grows, never shrinks)
void *osg_scratch(osg_ctx *ctx, int slot, size_t bytes);
void *osg_pinned(osg_ctx *ctx, size_t bytes);
// Host <-> device copies between a device buffer and the context's pinned staging buffer
// (osg_pinned), enqueued on ctx->stream.  Up to OSG_KCOPY_MAX bytes they run as a copy kernel in the
// stream's own compute queue, the GPU reading / writing the pinned pages over PCIe; larger ones, and
// host pointers outside the staging buffer, go to hipMemcpyAsync (the copy engines).
#define OSG_KCOPY_MAX (size_t(4) << 20)
int osg_upload(osg_ctx *ctx, void *dst_dev, const void *src_pinned, size_t bytes);
int osg_download(osg_ctx *ctx, void *dst_pinned, const void *src_dev, size_t bytes);
// Wait for everything enqueued on ctx->stream: an event recorded behind it, polled with
// hipEventQuery (a one-frame call returns within ~1 us of its last kernel instead of a blocking
// synchronisation's wake-up)
int osg_wait(osg_ctx *ctx);
// Before reusing the pinned block: nothing left on the stream.  A query first — a call that ended in
// osg_wait left the stream idle, and a synchronisation of an idle stream measured up to 14 us.
int osg_idle(osg_ctx *ctx);

#define OSG_HIP_CHECK(ctx, expr)                                                             \
    do {                                                                                     \
        hipError_t _e = (expr);                                                              \
        if (_e != hipSuccess)                                                                \
            return osg_set_error((ctx), OSG_E_HIP, "%s failed: %s (%s:%d)", #expr,          \
                                 hipGetErrorString(_e), __FILE__, __LINE__);                 \
    } while (0)

// propagate a negative OSG_E_* code
#define OSG_RC(expr)                                                                         \
    do {                                                                                     \
        const int _rc = (expr);                                                              \
        if (_rc < 0) return _rc;                                                             \
    } while (0)

#define OSG_REQUIRE(ctx, cond, ...)                                                          \
    do {                                                                                     \
        if (!(cond)) return osg_set_error((ctx), OSG_E_INVALID, __VA_ARGS__);               \
    } while (0)

#define OSG_ALLOC(ctx, ptr, slot, bytes)                                                     \
    do {                                                                                     \
        ptr = (decltype(ptr))osg_scratch((ctx), (slot), (bytes));                            \
        if (!(ptr)) return osg_set_error((ctx), OSG_E_NOMEM, "scratch alloc %zu B failed",  \
                                         (size_t)(bytes));                                   \
    } while (0)

// frame view validation (match.hip): array presence, grids index [0, n_cam), octaves in [0, 128)
int osg_check_frame(osg_ctx *ctx, const osg_frame *F);

// internal device-pointer launchers shared between translation units
int osg_launch_top2(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                    void *d_out);
// frame-batched top-2 on the I8 matrix cores (hamming_mfma.hip); 1 <= nt <= osg_top2_mfma_max_rows()
int osg_top2_mfma_max_rows();
int osg_launch_top2_batch_mfma(osg_ctx *ctx, const void *d_query, int32_t nq, const void *d_train, int32_t nt,
                               int32_t nb, void *d_out);
// the batched ORB extractor's stages (pyramid.hip, fast.hip), called by osg_orb_extract_batch (orb.hip)
int osg_pyramid_batch(osg_ctx *ctx, const uint8_t *d_images, int64_t img_bstride, int32_t rows, int32_t cols,
                      int32_t step, int32_t B, int32_t n_levels, const float *inv_scale, uint8_t *dev_out,
                      int64_t out_bstride, int64_t dev_bytes);
int osg_detect_batch(osg_ctx *ctx, const osg_image_pyramid *raw0, int32_t B, int64_t pyr_bstride, int32_t ini_th_fast,
                     int32_t min_th_fast, const int32_t *n_features_per_level, const float *scale_factors,
                     int32_t capacity, float *x, float *y, float *response, float *size, int32_t *level_start);

// ---- host worker threads -------------------------------------------------------------------------
// CPUs this process may run on at once: the smallest of the hardware threads, the affinity mask and
// the cgroup CPU quota (a GPU box's container sees every core of the host but is granted a share),
// divided between torchrun's local ranks (LOCAL_WORLD_SIZE); OSG_HOST_THREADS overrides.  Cached
// after the first call.
int osg_host_cpus();
// One process-wide pool of osg_host_cpus() - 1 persistent worker threads, shared by every context's
// host phases: concurrent callers (one per host thread driving its own context) queue their loops on
// the same workers instead of starting threads of their own, so the CPUs are not oversubscribed and a
// worker's thread_local buffers (the octree's nodes) survive from call to call.  The caller runs
// indices of its own loop too, so a loop finishes even when every worker is busy elsewhere.
// fn(arg, i) for i in [0, n) on the caller plus up to max_threads - 1 workers, indices handed out one
// at a time (the per-index work is independent; the order of completion is not).
void osg_parallel_run(int n, int max_threads, void (*fn)(void *, int), void *arg);
template <class F>
void osg_parallel_for(int n, int max_threads, F &&f)
{
    if (n <= 0) return;
    using Fn = typename std::remove_reference<F>::type;
    osg_parallel_run(n, max_threads, [](void *a, int i) { (*static_cast<Fn *>(a))(i); },
                     const_cast<void *>(static_cast<const void *>(&f)));
}
