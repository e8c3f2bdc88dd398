/* oracle_pyramid.c — TEST INFRASTRUCTURE ONLY (never linked into the product library).
 *
 * CPU restatement of ORBextractor::ComputePyramid (ref:src/ORBextractor.cc:1692-1743) and of the
 * GaussianBlur(workingMat, Size(7, 7), 2, 2, BORDER_REFLECT_101) of ORBextractor::operator()
 * (ref:src/ORBextractor.cc:1628-1636).  Both steps are OpenCV calls whose code is not in the
 * reference tree (OpenCV >= 4.4, ref:CMakeLists.txt); their published algorithms are restated here,
 * so parity with OpenCV itself is UNPINNED.  What is restated:
 *   - level size: cvRound((float)cols * mvInvScaleFactor[l]), same for rows (:1697);
 *   - cv::resize INTER_LINEAR on 8U (imgproc/resize.cpp, generic fixed-point path, no IPP):
 *     coefficient tables fx = (float)((dx + 0.5) * scale_x - 0.5), sx = floor, 11-bit short weights
 *     saturate_cast<short>((1 - fx) * 2048), saturate_cast<short>(fx * 2048); x clamped at the
 *     borders (sx < 0 -> 0 with fx = 0; sx >= w - 1 -> w - 1 with fx = 0, the columns from xmax on
 *     take S[sx] * 2048), rows clipped; horizontal pass exact in int; vertical pass
 *     (S0 b0 + S1 b1 + 2^21) >> 22 (FixedPtCast), except the columns the 128-bit universal-intrinsic
 *     VResizeLinearVec_32s8u covers (16-wide while x <= w - 16, then 8-wide while x < w - 8), which
 *     compute ((mulhi(S0 >> 4, b0) + mulhi(S1 >> 4, b1) + 2) >> 2) saturated;
 *   - copyMakeBorder(EDGE_THRESHOLD = 19 on every side, BORDER_REFLECT_101) of each level (:1717,
 *     :1738): borderInterpolate's reflect-101 loop on both axes;
 *   - GaussianBlur on 8U, OpenCV's bit-exact fixed-point path (smooth.dispatch.cpp,
 *     GaussianBlurFixedPoint): kernel from getGaussianKernelBitExact (exp(-x^2 / (2 sigma^2)) over
 *     x = -3..3, normalised) quantised to 8 fraction bits with getGaussianKernelFixedPoint_ED's error
 *     diffusion ([18 34 48 56 48 34 18] for 7 / sigma 2); rows then columns, both exact integer
 *     sums; result (sum + 2^15) >> 16; BORDER_REFLECT_101 on the level (the clone, :1628).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum { EDGE = 19 };

static int reflect101(int p, int len)
{
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - 2 - p;
    return p;
}

static int32_t sat_short(float v)
{
    long r = lrintf(v); /* cvRound: nearest, ties to even */
    return r < -32768 ? -32768 : r > 32767 ? 32767 : (int32_t)r;
}

static uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v); }

int64_t oracle_pyramid_layout(int32_t rows, int32_t cols, int32_t n_levels, const float *inv_scale, int32_t *lrows,
                              int32_t *lcols, int64_t *bordered_off, int64_t *blurred_off)
{
    int64_t at = 0;
    for (int l = 0; l < n_levels; l++) {
        lcols[l] = (int32_t)lrintf((float)cols * inv_scale[l]);
        lrows[l] = (int32_t)lrintf((float)rows * inv_scale[l]);
        bordered_off[l] = at;
        at += ((int64_t)(lrows[l] + 2 * EDGE) * (lcols[l] + 2 * EDGE) + 255) & ~(int64_t)255;
    }
    for (int l = 0; l < n_levels; l++) {
        blurred_off[l] = at;
        at += ((int64_t)lrows[l] * lcols[l] + 255) & ~(int64_t)255;
    }
    return at;
}

void oracle_gaussian_kernel7(int32_t k[7])
{
    /* getGaussianKernelBitExact(n = 7, sigma = 2): t_i = exp(x^2 * (-0.125 / sigma^2)), x = -6, -4, -2 */
    const double sigma = 2.0, scale2X = -0.125 / (sigma * sigma);
    double v[3], sum = 0;
    for (int i = 0, x = -6; i < 3; i++, x += 2) {
        v[i] = exp((double)(x * x) * scale2X);
        sum += v[i];
    }
    sum = sum * 2 + 1;
    const double mul1 = 1.0 / sum;
    /* getGaussianKernelFixedPoint_ED, 8 fraction bits */
    double err = 0;
    int64_t s = 0;
    for (int i = 0; i < 3; i++) {
        const double adj = v[i] * mul1 * 256.0 + err;
        const int64_t v0 = (int64_t)lrint(adj);
        err = adj - (double)v0;
        k[i] = k[6 - i] = (int32_t)v0;
        s += v0;
    }
    k[3] = (int32_t)(256 - 2 * s);
}

/* cv::resize(src, dst, Size(dw, dh), 0, 0, INTER_LINEAR), 8U, one channel */
static void resize_linear(const uint8_t *src, int sstep, int sw, int sh, uint8_t *dst, int dstep, int dw, int dh)
{
    const double scale_x = 1.0 / ((double)dw / sw), scale_y = 1.0 / ((double)dh / sh);
    int xofs[8192], xmax = dw;
    int16_t alpha[2 * 8192];
    for (int dx = 0; dx < dw; dx++) {
        float fx = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(fx);
        fx -= (float)sx;
        if (sx < 0) fx = 0, sx = 0;
        if (sx + 1 >= sw) {
            if (dx < xmax) xmax = dx;
            if (sx >= sw - 1) fx = 0, sx = sw - 1;
        }
        xofs[dx] = sx;
        alpha[2 * dx] = (int16_t)sat_short((1.f - fx) * 2048);
        alpha[2 * dx + 1] = (int16_t)sat_short(fx * 2048);
    }
    int xv = 0; /* columns of VResizeLinearVec_32s8u */
    while (xv <= dw - 16) xv += 16;
    while (xv < dw - 8) xv += 8;
    int D[2][8192];
    for (int dy = 0; dy < dh; dy++) {
        float fy = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)floorf(fy);
        fy -= (float)sy;
        const int b0 = sat_short((1.f - fy) * 2048), b1 = sat_short(fy * 2048);
        for (int k = 0; k < 2; k++) {
            int r = sy + k;
            r = r < 0 ? 0 : r >= sh ? sh - 1 : r;
            const uint8_t *S = src + (int64_t)r * sstep;
            for (int dx = 0; dx < dw; dx++)
                D[k][dx] = dx < xmax ? S[xofs[dx]] * alpha[2 * dx] + S[xofs[dx] + 1] * alpha[2 * dx + 1]
                                     : S[xofs[dx]] * 2048;
        }
        uint8_t *o = dst + (int64_t)dy * dstep;
        for (int dx = 0; dx < dw; dx++) {
            if (dx < xv) {
                const int m0 = ((D[0][dx] >> 4) * b0) >> 16, m1 = ((D[1][dx] >> 4) * b1) >> 16;
                o[dx] = sat_u8((m0 + m1 + 2) >> 2);
            } else {
                o[dx] = sat_u8((D[0][dx] * b0 + D[1][dx] * b1 + (1 << 21)) >> 22);
            }
        }
    }
}

int64_t oracle_orb_pyramid(const uint8_t *image, int32_t rows, int32_t cols, int32_t step, int32_t n_levels,
                           const float *inv_scale, uint8_t *out, int32_t blur)
{
    int32_t lr[64], lc[64];
    int64_t bo[64], bl[64];
    if (n_levels < 1 || n_levels > 64) return -1;
    const int64_t total = oracle_pyramid_layout(rows, cols, n_levels, inv_scale, lr, lc, bo, bl);
    for (int l = 0; l < n_levels; l++) {
        const int w = lc[l], h = lr[l], bstep = w + 2 * EDGE;
        if (w > 8192 || (l > 0 && lc[l - 1] > 8192)) return -1;
        uint8_t *B = out + bo[l];
        uint8_t *roi = B + (int64_t)EDGE * bstep + EDGE;
        if (l == 0) {
            for (int y = 0; y < h; y++) memcpy(roi + (int64_t)y * bstep, image + (int64_t)y * step, (size_t)w);
        } else {
            const int pw = lc[l - 1], ph = lr[l - 1], pstep = pw + 2 * EDGE;
            const uint8_t *proi = out + bo[l - 1] + (int64_t)EDGE * pstep + EDGE;
            resize_linear(proi, pstep, pw, ph, roi, bstep, w, h);
        }
        /* copyMakeBorder: the interior is in place; every border pixel reads its reflected pixel */
        for (int by = 0; by < h + 2 * EDGE; by++)
            for (int bx = 0; bx < w + 2 * EDGE; bx++) {
                const int y = by - EDGE, x = bx - EDGE;
                if (y >= 0 && y < h && x >= 0 && x < w) continue;
                B[(int64_t)by * bstep + bx] = roi[(int64_t)reflect101(y, h) * bstep + reflect101(x, w)];
            }
    }
    if (!blur) return total;
    int32_t k[7];
    oracle_gaussian_kernel7(k);
    for (int l = 0; l < n_levels; l++) {
        const int w = lc[l], h = lr[l], bstep = w + 2 * EDGE;
        const uint8_t *roi = out + bo[l] + (int64_t)EDGE * bstep + EDGE;
        uint8_t *o = out + bl[l];
        /* rows first: ufixedpoint16 sums (<= 255 * 256, exact) of the whole level */
        uint16_t *H = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)w * h);
        int *xi = (int *)malloc(sizeof(int) * (size_t)(w + 6));
        if (!H || !xi) {
            free(H);
            free(xi);
            return -1;
        }
        for (int j = 0; j < w + 6; j++) xi[j] = reflect101(j - 3, w);
        for (int y = 0; y < h; y++) {
            const uint8_t *r = roi + (int64_t)y * bstep;
            for (int x = 0; x < w; x++) {
                uint32_t s = 0;
                for (int t = 0; t < 7; t++) s += (uint32_t)r[xi[x + t]] * (uint32_t)k[t];
                H[(size_t)y * w + x] = (uint16_t)s;
            }
        }
        /* then columns (ufixedpoint32, exact) and one rounding */
        for (int y = 0; y < h; y++) {
            const uint16_t *hr[7];
            for (int t = 0; t < 7; t++) hr[t] = H + (size_t)reflect101(y + t - 3, h) * w;
            for (int x = 0; x < w; x++) {
                uint32_t acc = 0;
                for (int t = 0; t < 7; t++) acc += (uint32_t)hr[t][x] * (uint32_t)k[t];
                o[(int64_t)y * w + x] = (uint8_t)((acc + (1u << 15)) >> 16);
            }
        }
        free(H);
        free(xi);
    }
    return total;
}
