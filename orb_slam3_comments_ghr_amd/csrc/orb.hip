// orb.hip — ORBextractor's per-keypoint stages on gfx950: IC_Angle (ref:src/ORBextractor.cc:89-136)
// and computeOrbDescriptor (ref:src/ORBextractor.cc:148-208), for the keypoints of every level of
// one frame in one launch each.
//  * k_orb_angle — one wave per keypoint; lane u + 15 (u = -15..15) owns column u of the circular
//    patch: u I(u, 0) + sum over v = 1..15 with |u| <= umax[v] of u (I(u, v) + I(u, -v)) for m_10
//    and v (I(u, v) - I(u, -v)) for m_01, its 31 loads issued together (masked, not branched).  Integer sums, so the wave reduction equals the
//    reference's row-major order exactly; lane 0 evaluates fastAtan2.
//  * host: a = cosf(angle factorPI), b = sinf(angle factorPI) — the reference's std::cos(float) /
//    std::sin(float) from the same libm, so the rotated pattern rounds identically.
//  * k_orb_desc — one thread per (keypoint, descriptor byte), 8 keypoints per 256-thread
//    workgroup; the 512-point pattern staged in LDS; bit j = I(p[2j]) < I(p[2j+1]) at the rotated,
//    rint-rounded offsets (cvRound) around the rounded centre, addressed as the reference does in its
//    continuous blurred clone (a point left of column 0 reads the previous row's end).  A read outside
//    the whole level buffer (the reference reads whatever heap lies there) yields 0, and the call
//    returns how many keypoints did that.
// The argument block (level pointers and sizes, ~1.4 KB) travels as the kernel argument, not as a
// device copy the waves would first have to load.  Built with -ffp-contract=off: the rotation is two
// float products and a sum, as written.
#include <algorithm>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstring>
#include <vector>

#include "match_common.h"

#define GLOBAL __attribute__((address_space(1)))

namespace {

constexpr int HALF_PATCH = 15;
constexpr int MAX_LEVELS = 32;
constexpr int NPOINTS = 512;

struct OrbArgs {
    int n;
    GLOBAL const float *x, *y;
    GLOBAL const int32_t *level;
    GLOBAL const int32_t *pattern;               // 2 * NPOINTS
    GLOBAL const uint8_t *raw[MAX_LEVELS];
    GLOBAL const uint8_t *blur[MAX_LEVELS];
    int raw_rows[MAX_LEVELS], raw_cols[MAX_LEVELS], raw_step[MAX_LEVELS];
    int blur_rows[MAX_LEVELS], blur_cols[MAX_LEVELS], blur_step[MAX_LEVELS];  // step == cols
    int umax[HALF_PATCH + 1];
    GLOBAL float *angle;                         // n
    GLOBAL const float *cs;                      // 2n: (cos, sin)
    GLOBAL uint32_t *desc;                       // 8n words = 32n bytes
    GLOBAL int32_t *bad;                         // keypoints that read outside their level's buffer
    GLOBAL const int32_t *img;                   // batch: per keypoint its image (null: image 0)
    long long raw_bstride, blur_bstride;         // batch: bytes between the images' levels
};

__device__ __forceinline__ float fast_atan2(float y, float x)
{
    // OpenCV's cv::fastAtan2 (not in the reference tree): the same restatement as the oracle
    const float r2d = (float)(180 / 3.1415926535897932384626433832795);
    const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d;
    const float p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__global__ __launch_bounds__(256) void k_orb_angle(const OrbArgs A)
{
    const int lane = threadIdx.x & 63;
    const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (k >= A.n) return;
    const int l = A.level[k];
    const int cx = (int)rintf(A.x[k]), cy = (int)rintf(A.y[k]);
    const int step = A.raw_step[l];
    const long long bi = A.img ? A.img[k] : 0;
    GLOBAL const uint8_t *c = A.raw[l] + bi * A.raw_bstride + (size_t)cy * step + cx;
    // every read of the +-15 box is in bounds (checked on the host), so all 31 loads of a lane are
    // issued unconditionally and masked; lanes 31..63 read the centre column with weight 0
    const bool act = lane <= 2 * HALF_PATCH;
    const int u = act ? lane - HALF_PATCH : 0;
    const int au = u < 0 ? -u : u;
    int m10 = act ? u * (int)c[u] : 0, m01 = 0;
#pragma unroll
    for (int v = 1; v <= HALF_PATCH; v++) {
        const int p = c[u + v * step], m = c[u - v * step];
        const int w = (act && au <= A.umax[v]) ? 1 : 0;
        m01 += w * v * (p - m);
        m10 += w * u * (p + m);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        m10 += __shfl_xor(m10, o);
        m01 += __shfl_xor(m01, o);
    }
    if (lane == 0) A.angle[k] = fast_atan2((float)m01, (float)m10);
}

__global__ __launch_bounds__(256) void k_orb_desc(const OrbArgs A)
{
    __shared__ int2 s_pat[NPOINTS];
    for (int i = threadIdx.x; i < NPOINTS; i += 256)
        s_pat[i] = make_int2(A.pattern[2 * i], A.pattern[2 * i + 1]);
    __syncthreads();
    const int k = blockIdx.x * 8 + (threadIdx.x >> 5);
    const int byte = threadIdx.x & 31;
    if (k >= A.n) return;
    const int l = A.level[k];
    const int cx = (int)rintf(A.x[k]), cy = (int)rintf(A.y[k]);
    const float a = A.cs[2 * k], b = A.cs[2 * k + 1];
    // the reference reads a continuous clone (step = cols): a point past a row end wraps to the next row
    const int cols = A.blur_cols[l];
    const long long size = (long long)A.blur_rows[l] * cols;
    const long long c0 = (long long)cy * cols + cx;
    GLOBAL const uint8_t *img = A.blur[l] + (A.img ? A.img[k] : 0) * A.blur_bstride;
    uint32_t val = 0;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        int t[2];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int2 p = s_pat[16 * byte + 2 * j + s];
            const float px = (float)p.x, py = (float)p.y;
            const int dy = (int)rintf(px * b + py * a);
            const int dx = (int)rintf(px * a - py * b);
            const long long off = c0 + (long long)dy * cols + dx;
            const bool in = off >= 0 && off < size;
            bad |= !in;
            t[s] = in ? (int)img[off] : 0;  // outside the buffer: 0 (the reference reads foreign heap)
        }
        val |= (uint32_t)(t[0] < t[1]) << j;
    }
    // keypoints that read outside their level's buffer: one count per keypoint (its 32 lanes)
    const unsigned long long m = __ballot(bad);
    if (byte == 0 && ((m >> (threadIdx.x & 32)) & 0xffffffffull)) atomicAdd((int32_t *)A.bad, 1);
    // 4 bytes per word: lanes 4w..4w+3 of a keypoint's 32 build word w
    val <<= 8 * (byte & 3);
    val |= __shfl_xor(val, 1);
    val |= __shfl_xor(val, 2);
    if ((byte & 3) == 0) A.desc[8 * k + (byte >> 2)] = val;
}

template <typename T>
void set_off(T *&field, size_t off)
{
    field = (off == SIZE_MAX) ? nullptr : (T *)(uintptr_t)(off + 1);
}
template <typename T>
void relocate(T *&field, char *base)
{
    if (field) field = (T *)(base + ((uintptr_t)field - 1));
}

int check_pyr(osg_ctx *ctx, const osg_image_pyramid *P, int n_levels, const char *which)
{
    OSG_REQUIRE(ctx, P && P->n_levels >= n_levels && P->n_levels <= MAX_LEVELS && P->data && P->rows && P->cols &&
                         P->step,
                "%s pyramid needs %d levels (at most %d)", which, n_levels, MAX_LEVELS);
    for (int l = 0; l < n_levels; l++)
        OSG_REQUIRE(ctx, P->data[l] && P->rows[l] > 0 && P->cols[l] > 0 && P->step[l] >= P->cols[l],
                    "%s level %d", which, l);
    return OSG_OK;
}

// one side's levels into args: device pyramids read in place, host ones packed row-contiguous
void add_levels(osg_packer &pk, const osg_image_pyramid *P, int n_levels, std::vector<std::vector<uint8_t>> &keep,
                GLOBAL const uint8_t **img, int *rows, int *cols, int *step)
{
    for (int l = 0; l < n_levels; l++) {
        rows[l] = P->rows[l];
        cols[l] = P->cols[l];
        if (P->on_device) {
            img[l] = (GLOBAL const uint8_t *)P->data[l];
            step[l] = P->step[l];
            continue;
        }
        step[l] = cols[l];
        if (P->step[l] == cols[l]) {
            set_off(img[l], pk.add(P->data[l], (size_t)rows[l] * cols[l]));
        } else {
            keep.emplace_back((size_t)rows[l] * cols[l]);
            std::vector<uint8_t> &buf = keep.back();
            for (int r = 0; r < rows[l]; r++)
                std::memcpy(&buf[(size_t)r * cols[l]], P->data[l] + (size_t)r * P->step[l], cols[l]);
            set_off(img[l], pk.add(buf.data(), buf.size()));
        }
    }
}

// kimg (batch): per keypoint its image, whose device levels lie at raw / blurred's pointers + image x
// raw_bstride / blur_bstride
int orb_run(osg_ctx *ctx, const osg_image_pyramid *raw, const osg_image_pyramid *blurred, const osg_orb_keypoints *K,
            const int32_t *pattern, const int32_t *umax, int compute_angle, float *angle, uint8_t *desc,
            const int32_t *kimg = nullptr, int64_t raw_bstride = 0, int64_t blur_bstride = 0)
{
    if (!ctx) return OSG_E_INVALID;
    OSG_REQUIRE(ctx, K && K->n >= 0, "keypoints");
    const int n = K->n;
    if (n == 0) return OSG_OK;
    OSG_REQUIRE(ctx, K->x && K->y && K->level && pattern && angle && desc, "null argument");
    OSG_REQUIRE(ctx, !compute_angle || umax, "umax needed for the angles");
    int n_levels = 0;
    for (int k = 0; k < n; k++) {
        OSG_REQUIRE(ctx, K->level[k] >= 0 && K->level[k] < MAX_LEVELS, "keypoint %d: level %d", k, K->level[k]);
        OSG_REQUIRE(ctx, std::isfinite(K->x[k]) && std::isfinite(K->y[k]) && std::fabs(K->x[k]) < 1e8f &&
                             std::fabs(K->y[k]) < 1e8f,
                    "keypoint %d: coordinates", k);
        n_levels = std::max(n_levels, K->level[k] + 1);
    }
    int rc = check_pyr(ctx, blurred, n_levels, "blurred");
    if (rc < 0) return rc;
    if (blurred->on_device)
        for (int l = 0; l < n_levels; l++)
            OSG_REQUIRE(ctx, blurred->step[l] == blurred->cols[l],
                        "blurred level %d on the device must be continuous (step == cols), like the reference's clone", l);
    OrbArgs A{};
    A.n = n;
    osg_packer pk;
    std::vector<std::vector<uint8_t>> keep;
    keep.reserve(2 * MAX_LEVELS);
    if (compute_angle) {
        rc = check_pyr(ctx, raw, n_levels, "raw");
        if (rc < 0) return rc;
        for (int v = 0; v <= HALF_PATCH; v++)
            OSG_REQUIRE(ctx, umax[v] >= 0 && umax[v] <= HALF_PATCH, "umax[%d] = %d", v, umax[v]);
        for (int v = 0; v <= HALF_PATCH; v++) A.umax[v] = umax[v];
        // IC_Angle reads the (2 * 15 + 1)^2 box around the rounded centre
        for (int k = 0; k < n; k++) {
            const int l = K->level[k];
            const int cx = (int)std::rint(K->x[k]), cy = (int)std::rint(K->y[k]);
            OSG_REQUIRE(ctx, cx >= HALF_PATCH && cy >= HALF_PATCH && cx + HALF_PATCH < raw->cols[l] &&
                                 cy + HALF_PATCH < raw->rows[l],
                        "keypoint %d: the orientation patch leaves level %d", k, l);
        }
        add_levels(pk, raw, n_levels, keep, A.raw, A.raw_rows, A.raw_cols, A.raw_step);
    }
    add_levels(pk, blurred, n_levels, keep, A.blur, A.blur_rows, A.blur_cols, A.blur_step);
    set_off(A.x, pk.add(K->x, sizeof(float) * n));
    set_off(A.y, pk.add(K->y, sizeof(float) * n));
    set_off(A.level, pk.add(K->level, sizeof(int32_t) * n));
    if (kimg) {
        OSG_REQUIRE(ctx, raw->on_device && blurred->on_device, "batched keypoints need device pyramids");
        set_off(A.img, pk.add(kimg, sizeof(int32_t) * n));
        A.raw_bstride = raw_bstride;
        A.blur_bstride = blur_bstride;
    }
    set_off(A.pattern, pk.add(pattern, sizeof(int32_t) * 2 * NPOINTS));
    const size_t in_bytes = (pk.total + 255) & ~size_t(255);
    // outputs / exchange: angle n | cs 2n | bad 1 (256-aligned) | desc 32n
    const size_t o_cs = ((size_t)n * 4 + 255) & ~size_t(255);
    const size_t o_bad = o_cs + (((size_t)n * 8 + 255) & ~size_t(255));
    const size_t o_desc = o_bad + 256;
    const size_t out_bytes = o_desc + (size_t)n * 32;
    char *pin = (char *)osg_pinned(ctx, in_bytes + out_bytes + 256);
    if (!pin) return osg_set_error(ctx, OSG_E_NOMEM, "pinned alloc failed");
    OSG_RC(osg_idle(ctx));  // the pinned block may still be in use
    pk.fill_parallel(pin, 8);
    char *pin_out = pin + in_bytes;
    char *dev_in = nullptr, *dev_out = nullptr;
    OSG_ALLOC(ctx, dev_in, SLOT_TMP0, pk.total + 256);
    OSG_ALLOC(ctx, dev_out, SLOT_TMP2, out_bytes);
    relocate(A.x, dev_in);
    relocate(A.y, dev_in);
    relocate(A.level, dev_in);
    relocate(A.img, dev_in);
    relocate(A.pattern, dev_in);
    for (int l = 0; l < n_levels; l++) {
        if (compute_angle && !raw->on_device) relocate(A.raw[l], dev_in);
        if (!blurred->on_device) relocate(A.blur[l], dev_in);
    }
    A.angle = (GLOBAL float *)dev_out;
    A.cs = (GLOBAL const float *)(dev_out + o_cs);
    A.bad = (GLOBAL int32_t *)(dev_out + o_bad);
    A.desc = (GLOBAL uint32_t *)(dev_out + o_desc);
    *(int32_t *)(pin_out + o_bad) = 0;
    hipEvent_t *ev = osg_ctx_events(ctx);
    if (!ev) return osg_set_error(ctx, OSG_E_HIP, "event create failed");
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_in, pin, pk.total, hipMemcpyHostToDevice, ctx->stream));
    float ms_angle = 0.f;
    float *ang = (float *)pin_out;
    if (compute_angle) {
        OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
        hipLaunchKernelGGL(k_orb_angle, dim3((n + 3) / 4), dim3(256), 0, ctx->stream, A);
        OSG_HIP_CHECK(ctx, hipGetLastError());
        OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
        OSG_RC(osg_download(ctx, ang, dev_out, sizeof(float) * n));
        OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
        OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms_angle, ev[0], ev[1]));
    } else {
        std::memcpy(ang, angle, sizeof(float) * n);
    }
    // computeOrbDescriptor :153-154 — angle * factorPI, then std::cos(float) / std::sin(float)
    const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
    float *cs = (float *)(pin_out + o_cs);
    for (int k = 0; k < n; k++) {
        const float t = ang[k] * factorPI;
        cs[2 * k] = cosf(t);
        cs[2 * k + 1] = sinf(t);
    }
    OSG_HIP_CHECK(ctx, hipMemcpyAsync(dev_out + o_cs, cs, o_bad - o_cs + 256, hipMemcpyHostToDevice, ctx->stream));
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[0], ctx->stream));
    hipLaunchKernelGGL(k_orb_desc, dim3((n + 7) / 8), dim3(256), 0, ctx->stream, A);
    OSG_HIP_CHECK(ctx, hipGetLastError());
    OSG_HIP_CHECK(ctx, hipEventRecord(ev[1], ctx->stream));
    OSG_RC(osg_download(ctx, pin_out + o_bad, dev_out + o_bad, out_bytes - o_bad));
    OSG_HIP_CHECK(ctx, hipStreamSynchronize(ctx->stream));  // (a polled wait measured slower here)
    float ms_desc = 0.f;
    OSG_HIP_CHECK(ctx, hipEventElapsedTime(&ms_desc, ev[0], ev[1]));
    ctx->last_kernel_ms = ms_angle + ms_desc;
    if (compute_angle) std::memcpy(angle, ang, sizeof(float) * n);
    std::memcpy(desc, pin_out + o_desc, (size_t)n * 32);
    return *(int32_t *)(pin_out + o_bad);
}

}  // namespace

extern "C" {

// ORBextractor::operator() for B images: osg_pyramid_batch -> osg_detect_batch -> the batched
// describe (orb_run with per-keypoint images).  Same results as the three per-image calls.
int osg_orb_extract_batch(osg_ctx *ctx, const uint8_t *d_images, int64_t image_stride, int32_t rows, int32_t cols,
                          int32_t step, int32_t n_images, const osg_orb_extract_params *P, int32_t capacity, float *x,
                          float *y, float *angle, float *response, float *size, int32_t *octave, uint8_t *desc,
                          int32_t *counts)
{
    if (!ctx) return OSG_E_INVALID;
    static const bool prof = getenv("OSG_ORB_PROFILE") != nullptr;  // host phase times to stderr
    const auto tp0 = std::chrono::steady_clock::now();
    auto ms_since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp0).count(); };
    OSG_REQUIRE(ctx, n_images >= 0 && n_images <= 65535, "n_images = %d", n_images);
    if (n_images == 0) return 0;
    OSG_REQUIRE(ctx, d_images && P && P->scale_factors && P->inv_scale_factors && P->n_features_per_level &&
                         P->pattern && P->umax && counts && capacity >= 0,
                "null argument");
    OSG_REQUIRE(ctx, capacity == 0 || (x && y && angle && response && size && octave && desc), "null output");
    OSG_REQUIRE(ctx, step >= cols && (n_images == 1 || image_stride >= (int64_t)step * rows), "image step / stride");
    const int L = P->n_levels;
    OSG_REQUIRE(ctx, L >= 1 && L <= MAX_LEVELS, "n_levels = %d", L);
    int32_t lr[MAX_LEVELS], lc[MAX_LEVELS];
    int64_t bo[MAX_LEVELS], bl[MAX_LEVELS];
    const int64_t total = osg_orb_pyramid_layout(rows, cols, L, P->inv_scale_factors, lr, lc, bo, bl);
    OSG_REQUIRE(ctx, total > 0, "pyramid layout");
    const int64_t pstride = (total + 4095) & ~(int64_t)4095;
    uint8_t *pyr = nullptr;
    OSG_ALLOC(ctx, pyr, SLOT_TMP8, (size_t)pstride * n_images);
    OSG_RC(osg_pyramid_batch(ctx, d_images, image_stride, rows, cols, step, n_images, L, P->inv_scale_factors, pyr,
                             pstride, pstride * n_images));
    const uint8_t *rawp[MAX_LEVELS], *blp[MAX_LEVELS];
    int32_t rstep[MAX_LEVELS], bstep[MAX_LEVELS];
    for (int l = 0; l < L; l++) {
        rstep[l] = lc[l] + 38;
        rawp[l] = pyr + bo[l] + (int64_t)19 * rstep[l] + 19;
        bstep[l] = lc[l];
        blp[l] = pyr + bl[l];
    }
    const osg_image_pyramid raw0 = {L, 1, rawp, lr, lc, rstep};
    const osg_image_pyramid blur0 = {L, 1, blp, lr, lc, bstep};
    std::vector<int32_t> ls((size_t)n_images * (L + 1));
    const int n = osg_detect_batch(ctx, &raw0, n_images, pstride, P->ini_th_fast, P->min_th_fast,
                                   P->n_features_per_level, P->scale_factors, capacity, x, y, response, size, ls.data());
    if (n < 0) return n;
    const double t_detect = ms_since();
    // all images' keypoints in one list for the describe kernels, with their image and level
    std::vector<float> kx(n), ky(n), ka(n);
    std::vector<int32_t> kl(n), ki(n);
    std::vector<uint8_t> kd((size_t)n * 32);
    for (int b = 0, q = 0; b < n_images; b++) {
        const int32_t *lsb = ls.data() + (size_t)b * (L + 1);
        counts[b] = lsb[L];
        for (int l = 0; l < L; l++)
            for (int i = lsb[l]; i < lsb[l + 1]; i++, q++) {
                kx[q] = x[(size_t)b * capacity + i];
                ky[q] = y[(size_t)b * capacity + i];
                kl[q] = l;
                ki[q] = b;
                octave[(size_t)b * capacity + i] = l;
            }
    }
    const double t_list = ms_since();
    const osg_orb_keypoints K = {n, kx.data(), ky.data(), kl.data()};
    const int rc = orb_run(ctx, &raw0, &blur0, &K, P->pattern, P->umax, 1, ka.data(), kd.data(), ki.data(), pstride,
                           pstride);
    if (rc < 0) return rc;
    const double t_desc = ms_since();
    for (int b = 0, q = 0; b < n_images; b++)
        for (int i = 0; i < counts[b]; i++, q++) {
            angle[(size_t)b * capacity + i] = ka[q];
            std::memcpy(desc + ((size_t)b * capacity + i) * 32, kd.data() + (size_t)q * 32, 32);
        }
    if (prof)
        fprintf(stderr, "[osg orb extract] %d images, %d keypoints: pyramid + detect %.3f ms, list %.3f ms, describe %.3f ms, "
                        "scatter %.3f ms\n", n_images, n, t_detect, t_list - t_detect, t_desc - t_list, ms_since() - t_desc);
    return n;
}

int osg_orb_describe(osg_ctx *ctx, const osg_image_pyramid *raw, const osg_image_pyramid *blurred,
                     const osg_orb_keypoints *K, const int32_t *pattern, const int32_t *umax, int32_t compute_angle,
                     float *angle, uint8_t *desc)
{
    return orb_run(ctx, raw, blurred, K, pattern, umax, compute_angle, angle, desc);
}

}  // extern "C"
