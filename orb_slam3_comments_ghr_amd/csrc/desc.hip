// desc.hip — MapPoint::ComputeDistinctiveDescriptors on gfx950 (ref:src/MapPoint.cc:444-535).
//
// For each MapPoint: the N descriptors of its observations (left and right rows per keyframe, in
// the caller's std::map order), all pairwise DescriptorDistances, and the index whose sorted
// distance row has the smallest element [0.5 * (N - 1)] (the "median", self-distance 0 included;
// strict '<' so the first index wins ties).  LocalMapping runs it for every MapPoint of a keyframe
// (ref:src/LocalMapping.cc:1066-1082, :421-436), so the entry point takes a whole list.
//
// One wave per MapPoint, lane = row.  The row's k-th smallest distance (k = floor((N-1)/2)) is found
// by a 9-step binary search over the distance value (0..256): count(d <= v) >= k + 1.  Each step
// recomputes the row's distances against descriptors that are wave-uniform (scalar loads), which
// beats keeping N distances per lane in LDS for the N (2..~30) the reference sees.  The wave then
// takes min over (median << 16 | row).
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int DW = 256;           // threads per workgroup: 4 MapPoints
constexpr int MP_PER_WG = DW / 64;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc)
{
    uint32_t r;
    asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
    return r;
}

__device__ __forceinline__ uint32_t dist8(const u32x4 &a0, const u32x4 &a1, const u32x4 &b0, const u32x4 &b1)
{
    uint32_t d = __popc(a0.x ^ b0.x);
    d = bcnt_acc(a0.y ^ b0.y, d);
    d = bcnt_acc(a0.z ^ b0.z, d);
    d = bcnt_acc(a0.w ^ b0.w, d);
    d = bcnt_acc(a1.x ^ b1.x, d);
    d = bcnt_acc(a1.y ^ b1.y, d);
    d = bcnt_acc(a1.z ^ b1.z, d);
    d = bcnt_acc(a1.w ^ b1.w, d);
    return d;
}

__global__ __launch_bounds__(DW) void k_distinctive(GLOBAL const u32x4 *__restrict__ desc,
                                                    GLOBAL const int32_t *__restrict__ start, int n_points,
                                                    GLOBAL int32_t *__restrict__ best_idx)
{
    const int p = __builtin_amdgcn_readfirstlane(blockIdx.x * MP_PER_WG + (int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (p >= n_points) return;
    const int base = __builtin_amdgcn_readfirstlane(start[p]);
    const int N = __builtin_amdgcn_readfirstlane(start[p + 1]) - base;
    if (N <= 0) {
        if (lane == 0) best_idx[p] = -1;
        return;
    }
    GLOBAL const u32x4 *D = desc + 2 * (size_t)base;
    const int k = (N - 1) >> 1;  // (size_t)(0.5 * (N - 1)), ref:src/MapPoint.cc:514
    uint32_t key = 0xFFFFFFFFu;
    for (int i = lane; i < N + ((64 - N % 64) % 64); i += 64) {  // every lane runs the same trip count
        const bool live = i < N;
        const int ii = live ? i : 0;
        const u32x4 a0 = D[2 * ii], a1 = D[2 * ii + 1];
        int lo = 0, hi = 256;
        while (lo < hi) {  // uniform: 9 steps for every lane
            const int mid = (lo + hi) >> 1;
            int c = 0;
            for (int j = 0; j < N; j++) {
                const u32x4 b0 = D[2 * j], b1 = D[2 * j + 1];  // wave-uniform address
                c += (int)dist8(a0, a1, b0, b1) <= mid;
            }
            // only the row's own answer matters; the step is taken with the row's count
            if (c >= k + 1) hi = mid; else lo = mid + 1;
        }
        if (live) {
            const uint32_t kk = ((uint32_t)lo << 16) | (uint32_t)i;
            key = kk < key ? kk : key;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t other = __shfl_xor(key, o);
        key = other < key ? other : key;
    }
    if (lane == 0) best_idx[p] = (int32_t)(key & 0xFFFF);
}

int launch(osg_ctx *ctx, const void *d_desc, const void *d_start, int n_points, void *d_best)
{
    if (n_points == 0) return OSG_OK;
    hipLaunchKernelGGL(k_distinctive, dim3((n_points + MP_PER_WG - 1) / MP_PER_WG), dim3(DW), 0, ctx->stream,
                       (GLOBAL const u32x4 *)d_desc, (GLOBAL const int32_t *)d_start, n_points,
                       (GLOBAL int32_t *)d_best);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    return OSG_OK;
}

}  // namespace

extern "C" {

int osg_compute_distinctive_descriptors(osg_ctx *ctx, const uint8_t *desc, const int32_t *start, int32_t n_points,
                                        int32_t *best_idx)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, n_points >= 0 && (n_points == 0 || (start && best_idx)), "null argument / n_points");
    if (n_points == 0) return OSG_OK;
    OSG_REQUIRE(ctx, start[0] == 0, "start[0] must be 0");
    for (int p = 0; p < n_points; p++)
        OSG_REQUIRE(ctx, start[p + 1] >= start[p] && start[p + 1] - start[p] <= 65535,
                    "point %d: observation count %d out of range", p, start[p + 1] - start[p]);
    const size_t total = (size_t)start[n_points];
    OSG_REQUIRE(ctx, total == 0 || desc, "null descriptors");
    const size_t d_bytes = ((total * 32 + 255) & ~size_t(255)), s_bytes = ((sizeof(int32_t) * (n_points + 1) + 255) & ~size_t(255));
    const size_t o_bytes = sizeof(int32_t) * (size_t)n_points;
    char *pin = (char *)osg_pinned(ctx, d_bytes + s_bytes + o_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    if (total) std::memcpy(pin, desc, total * 32);
    std::memcpy(pin + d_bytes, start, sizeof(int32_t) * (n_points + 1));
    int32_t *pin_out = (int32_t *)(pin + d_bytes + s_bytes);
    char *dev = nullptr;
    OSG_ALLOC(ctx, dev, SLOT_TMP0, d_bytes + s_bytes + o_bytes + 256);
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev, pin, d_bytes + s_bytes, hipMemcpyHostToDevice, ctx->stream));
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    int rc = launch(ctx, dev, dev + d_bytes, n_points, dev + d_bytes + s_bytes);
    if (rc < 0) return rc;
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out, dev + d_bytes + s_bytes, o_bytes));
    OSG_RC(osg_wait(ctx));
    float ms = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms, ev[0], ev[1]));
    ctx->last_kernel_ms = ms;
    std::memcpy(best_idx, pin_out, o_bytes);
    return OSG_OK;
}

int osg_compute_distinctive_descriptors_dev(osg_ctx *ctx, const void *d_desc, const void *d_start, int32_t n_points,
                                            void *d_best_idx)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, n_points >= 0 && (n_points == 0 || (d_desc && d_start && d_best_idx)), "null argument");
    return launch(ctx, d_desc, d_start, n_points, d_best_idx);
}

}  // extern "C"
