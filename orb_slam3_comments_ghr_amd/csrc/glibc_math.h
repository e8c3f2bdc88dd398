// glibc_math.h — the host libm's float atan2f, restated for the device (and the host checker).
//
// The reference's KannalaBrandt8::project (ref:src/CameraModels/KannalaBrandt8.cpp:62-80) takes
// theta = atan2f(sqrtf(x^2 + y^2), z) and psi = atan2f(y, x) in float through the host libm.  The
// device library's atan2f differs from glibc's in the last bit now and then, and one ulp of theta
// moves a KB8 PoseOptimization off the reference's arithmetic.  glibc 2.35 on x86_64 evaluates
// atan2f with the float version of fdlibm's algorithm (sysdeps/ieee754/flt-32/e_atan2f.c over
// s_atanf.c, the Sun Microsystems code of 1993): quadrant rules on the bit patterns, y / x rounded
// to float, then atanf by a four-interval argument reduction and an 11-term odd polynomial split
// into two Horner chains.  Restated here from that published algorithm, in float, without
// contraction.  tools/glibc_math_check.cc compares it with the host's atan2f bit for bit (10^8+
// random and KB8-range arguments, plus every quadrant / zero / infinity case); tests/test_exact_math.py
// runs a sample of that check in the CPU suite.
#pragma once
#include <cmath>
#include <cstdint>
#include <cstring>

#ifdef __HIPCC__
#define OSG_GM_HD __host__ __device__
#else
#define OSG_GM_HD
#endif
#ifdef __clang__
#define OSG_GM_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define OSG_GM_NOCONTRACT
#endif

namespace osgm {

OSG_GM_HD inline int32_t f2i(float x)
{
    int32_t i;
    __builtin_memcpy(&i, &x, 4);
    return i;
}
OSG_GM_HD inline float i2f(int32_t i)
{
    float x;
    __builtin_memcpy(&x, &i, 4);
    return x;
}

// fdlibm float atanf (s_atanf.c).  The interval branches are evaluated branch-free: every lane forms
// the numerator / denominator of its interval's reduction with the same float operations and
// divides once (x / 1 = x exactly on the |x| < 0.4375 path), so a wave whose lanes fall into
// different intervals runs one division, not one per interval.
OSG_GM_HD inline float atanf_fd(float x)
{
    OSG_GM_NOCONTRACT
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    const int32_t hx = f2i(x);
    const int32_t ix = hx & 0x7fffffff;
    if (ix >= 0x4c000000) {  // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;  // NaN
        return hx > 0 ? 1.5707962513e+00f + 7.5497894159e-08f : -1.5707962513e+00f - 7.5497894159e-08f;
    }
    if (ix < 0x31000000) return x;  // |x| < 2^-29
    // id: -1 |x| < 0.4375; 0 7/16 <= |x| < 11/16; 1 11/16 <= |x| < 19/16; 2 |x| < 2.4375; 3 otherwise
    const int id = ix < 0x3ee00000 ? -1 : ix < 0x3f300000 ? 0 : ix < 0x3f980000 ? 1 : ix < 0x401c0000 ? 2 : 3;
    const float ax = fabsf(x);
    float num, den;
    if (id < 0) { num = x; den = 1.0f; }
    else if (id == 0) { num = 2.0f * ax - 1.0f; den = 2.0f + ax; }
    else if (id == 1) { num = ax - 1.0f; den = ax + 1.0f; }
    else if (id == 2) { num = ax - 1.5f; den = 1.0f + 1.5f * ax; }
    else { num = -1.0f; den = ax; }
    x = num / den;
    const float z = x * x;
    const float w = z * z;
    const float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    const float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    const float hi = id == 0 ? 4.6364760399e-01f : id == 1 ? 7.8539812565e-01f : id == 2 ? 9.8279368877e-01f : 1.5707962513e+00f;
    const float lo = id == 0 ? 5.0121582440e-09f : id == 1 ? 3.7748947079e-08f : id == 2 ? 3.4473217170e-08f : 7.5497894159e-08f;
    const float r = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -r : r;
}

// fdlibm float atan2f (e_atan2f.c)
OSG_GM_HD inline float atan2f_fd(float y, float x)
{
    OSG_GM_NOCONTRACT
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f, pi = 3.1415927410e+00f,
                pi_lo = -8.7422776573e-08f;
    const int32_t hx = f2i(x), ix = hx & 0x7fffffff;
    const int32_t hy = f2i(y), iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;  // NaN
    if (hx == 0x3f800000) return atanf_fd(y);               // x = 1.0
    const int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);      // 2 sign(x) + sign(y)
    if (iy == 0) {                                          // y = 0
        switch (m) {
        case 0:
        case 1: return y;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;  // x = 0
    if (ix == 0x7f800000) {                                       // x = inf
        if (iy == 0x7f800000) {
            switch (m) {
            case 0: return pi_o_4 + tiny;
            case 1: return -pi_o_4 - tiny;
            case 2: return 3.0f * pi_o_4 + tiny;
            default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
        case 0: return 0.0f;
        case 1: return -0.0f;
        case 2: return pi + tiny;
        default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;  // y = inf
    const int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;  // |y / x| > 2^60
    else if (hx < 0 && k < -60) z = 0.0f;   // |y| / x < -2^60
    else z = atanf_fd(fabsf(y / x));
    switch (m) {
    case 0: return z;
    case 1: return i2f(f2i(z) ^ (int32_t)0x80000000u);
    case 2: return pi - (z - pi_lo);
    default: return (z - pi_lo) - pi;
    }
}

}  // namespace osgm
