// exact_math.h — correctly rounded cube / sin / cos for the FP64 LM paths (pose.hip, ba.hip).
//
// The reference evaluates pow(theta, 3), sin(theta), cos(theta) (SE3Quat::exp,
// ref:Thirdparty/g2o/g2o/types/se3quat.h:223-257) and pow(2 rho - 1, 3) (the LM step-quality
// rule, ref:Thirdparty/g2o/g2o/core/optimization_algorithm_levenberg.cpp:134-140) through the
// host libm, whose last bit is platform-dependent (glibc 2.35 misrounds 0.06-0.09 % of these
// arguments; the device library differs from both).  Device and oracle therefore both evaluate
// the mathematical value correctly rounded: here in double-double arithmetic with one final
// rounding, in the oracle (oracle/oracle_ba.c) independently in __float128.  Both are checked
// against mpmath and against each other (tests/test_exact_math.py, tools/exact_math_check.cc).
// sin / cos use the series only on [0, 0.8] (the update magnitudes LM produces); larger
// arguments take the library function on either side.
//
// Every expression here relies on IEEE evaluation without contraction (a pragma in each body; the
// error-free products use explicit fma()).
#pragma once
#include <cmath>

#ifdef __HIPCC__
#define OSG_HD __host__ __device__
#else
#define OSG_HD
#endif
// no contraction inside the error-free transforms, whatever the translation unit's flags
#ifdef __clang__
#define OSGX_NOCONTRACT _Pragma("clang fp contract(off)")
#else
#define OSGX_NOCONTRACT
#endif

namespace osgx {

struct dd {
    double h, l;
};

OSG_HD inline dd two_sum(double a, double b)
{
    OSGX_NOCONTRACT
    const double s = a + b;
    const double bb = s - a;
    const double e = (a - (s - bb)) + (b - bb);
    return {s, e};
}
OSG_HD inline dd quick_two_sum(double a, double b)
{
    OSGX_NOCONTRACT
    const double s = a + b;
    return {s, b - (s - a)};
}
OSG_HD inline dd two_prod(double a, double b)
{
    OSGX_NOCONTRACT
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
OSG_HD inline dd dd_mul(dd a, dd b)
{
    OSGX_NOCONTRACT
    dd p = two_prod(a.h, b.h);
    p.l += a.h * b.l + a.l * b.h;
    return quick_two_sum(p.h, p.l);
}
OSG_HD inline dd dd_add(dd a, dd b)
{
    OSGX_NOCONTRACT
    dd s = two_sum(a.h, b.h);
    const dd t = two_sum(a.l, b.l);
    s.l += t.h;
    s = quick_two_sum(s.h, s.l);
    s.l += t.l;
    return quick_two_sum(s.h, s.l);
}

// t^3 rounded once (pow(t, 3) of a correctly rounding libm)
OSG_HD inline double cube_rn(double t)
{
    OSGX_NOCONTRACT
    const double p = t * t;
    const double q = p * t;
    if (!(fabs(q) < 1e300) || !(fabs(p) < 1e300) || q == 0.0) return q;  // inf / nan / overflow / zero
    const double pe = fma(t, t, -p);  // t^2 = p + pe exactly
    const double qe = fma(p, t, -q);  // p t = q + qe exactly
    return q + (qe + pe * t);
}

// Terms of the x^2 series that matter at x: the first K coefficients when the first dropped term,
// |c_K| x^(2K) (c_K = 1 / (2K)! or 1 / (2K + 1)!), is below 2^-118 of the leading 1 — far under the
// double-double rounding error of the sum (2^-104), so the final rounding is that of the full
// 15-term series.  LM rotation updates are mostly 1e-5 .. 1e-2 rad: 4 to 8 terms instead of 15.
OSG_HD inline int series_terms(double x)
{
    const double lim[14] = {2.4532694666933987e-18, 2.915197201209678e-09, 3.5972075921221558e-06,
                            0.00013661476184978878, 0.0012700544907879897, 0.0057973980883841278,
                            0.017547082534525357,   0.040967787164514206,  0.080299195873085955,
                            0.13906865564818396,    0.21990626161203589,   0.3245626875579769,
                            0.45402522493007225,    0.6086654061405502};
    int K = 15;
#pragma unroll
    for (int i = 13; i >= 0; i--)
        if (x < lim[i]) K = i + 1;
    return K;
}

// sin(x) / cos(x) for 0 <= x <= 0.8: Horner in double-double over x^2 from the series_terms(x)-th
// coefficient down (the branches are uniform when every lane holds the same x), one final rounding
OSG_HD inline double sin_rn_small(double x)
{
    OSGX_NOCONTRACT
    const dd c[15] = {{1.0, 0.0},
                      {-0.16666666666666666, -9.25185853854297e-18},
                      {0.008333333333333333, 1.1564823173178714e-19},
                      {-0.0001984126984126984, -1.7209558293420705e-22},
                      {2.7557319223985893e-06, -1.858393274046472e-22},
                      {-2.505210838544172e-08, 1.448814070935912e-24},
                      {1.6059043836821613e-10, 1.2585294588752098e-26},
                      {-7.647163731819816e-13, -7.03872877733453e-30},
                      {2.8114572543455206e-15, 1.6508842730861433e-31},
                      {-8.22063524662433e-18, -2.2141894119604265e-34},
                      {1.9572941063391263e-20, -1.3643503830087908e-36},
                      {-3.868170170630684e-23, 8.843177655482344e-40},
                      {6.446950284384474e-26, -1.9330404233703465e-42},
                      {-9.183689863795546e-29, -1.4303150396787322e-45},
                      {1.1309962886447716e-31, 1.0498015412959506e-47}};
    const dd x2 = two_prod(x, x);
    const int K = series_terms(x);
    dd s = c[14];
#pragma unroll
    for (int k = 13; k >= 0; k--) {
        if (k == K - 1) s = c[k];
        else if (k < K - 1) s = dd_add(dd_mul(s, x2), c[k]);
    }
    const dd r = dd_mul(s, dd{x, 0.0});
    return r.h + r.l;
}
OSG_HD inline double cos_rn_small(double x)
{
    OSGX_NOCONTRACT
    const dd c[15] = {{1.0, 0.0},
                      {-0.5, 0.0},
                      {0.041666666666666664, 2.3129646346357427e-18},
                      {-0.001388888888888889, 5.300543954373577e-20},
                      {2.48015873015873e-05, 2.1511947866775882e-23},
                      {-2.755731922398589e-07, -2.3767714622250297e-23},
                      {2.08767569878681e-09, -1.20734505911326e-25},
                      {-1.1470745597729725e-11, -2.0655512752830745e-28},
                      {4.779477332387385e-14, 4.399205485834081e-31},
                      {-1.5619206968586225e-16, -1.1910679660273754e-32},
                      {4.110317623312165e-19, 1.4412973378659527e-36},
                      {-8.896791392450574e-22, 7.911402614872376e-38},
                      {1.6117375710961184e-24, -3.6846573564509766e-41},
                      {-2.4795962632247976e-27, 1.2953730964765229e-43},
                      {3.279889237069838e-30, 1.5117542744029879e-46}};
    const dd x2 = two_prod(x, x);
    const int K = series_terms(x);
    dd s = c[14];
#pragma unroll
    for (int k = 13; k >= 0; k--) {
        if (k == K - 1) s = c[k];
        else if (k < K - 1) s = dd_add(dd_mul(s, x2), c[k]);
    }
    return s.h + s.l;
}
// sin and cos of one argument at once: the two Horner chains of sin_rn_small / cos_rn_small
// interleaved in one loop (the same operations on the same values, so the same two results), which
// lets a latency-bound caller (SE3 exp in the LM loops) overlap them.
OSG_HD inline void sincos_rn_small(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    const dd cs_[15] = {{1.0, 0.0},
                        {-0.16666666666666666, -9.25185853854297e-18},
                        {0.008333333333333333, 1.1564823173178714e-19},
                        {-0.0001984126984126984, -1.7209558293420705e-22},
                        {2.7557319223985893e-06, -1.858393274046472e-22},
                        {-2.505210838544172e-08, 1.448814070935912e-24},
                        {1.6059043836821613e-10, 1.2585294588752098e-26},
                        {-7.647163731819816e-13, -7.03872877733453e-30},
                        {2.8114572543455206e-15, 1.6508842730861433e-31},
                        {-8.22063524662433e-18, -2.2141894119604265e-34},
                        {1.9572941063391263e-20, -1.3643503830087908e-36},
                        {-3.868170170630684e-23, 8.843177655482344e-40},
                        {6.446950284384474e-26, -1.9330404233703465e-42},
                        {-9.183689863795546e-29, -1.4303150396787322e-45},
                        {1.1309962886447716e-31, 1.0498015412959506e-47}};
    const dd cc_[15] = {{1.0, 0.0},
                        {-0.5, 0.0},
                        {0.041666666666666664, 2.3129646346357427e-18},
                        {-0.001388888888888889, 5.300543954373577e-20},
                        {2.48015873015873e-05, 2.1511947866775882e-23},
                        {-2.755731922398589e-07, -2.3767714622250297e-23},
                        {2.08767569878681e-09, -1.20734505911326e-25},
                        {-1.1470745597729725e-11, -2.0655512752830745e-28},
                        {4.779477332387385e-14, 4.399205485834081e-31},
                        {-1.5619206968586225e-16, -1.1910679660273754e-32},
                        {4.110317623312165e-19, 1.4412973378659527e-36},
                        {-8.896791392450574e-22, 7.911402614872376e-38},
                        {1.6117375710961184e-24, -3.6846573564509766e-41},
                        {-2.4795962632247976e-27, 1.2953730964765229e-43},
                        {3.279889237069838e-30, 1.5117542744029879e-46}};
    const dd x2 = two_prod(x, x);
    const int K = series_terms(x);
    dd a = cs_[14], c = cc_[14];
#pragma unroll
    for (int k = 13; k >= 0; k--) {
        if (k == K - 1) {
            a = cs_[k];
            c = cc_[k];
        } else if (k < K - 1) {
            a = dd_add(dd_mul(a, x2), cs_[k]);
            c = dd_add(dd_mul(c, x2), cc_[k]);
        }
    }
    const dd r = dd_mul(a, dd{x, 0.0});
    sn = r.h + r.l;
    cs = c.h + c.l;
}
OSG_HD inline void sincos_ref(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    if (x >= 0.0 && x <= 0.8) {
        sincos_rn_small(x, sn, cs);
    } else {
        sn = sin(x);
        cs = cos(x);
    }
}
OSG_HD inline double sin_ref(double x)
{
    OSGX_NOCONTRACT
    return (x >= 0.0 && x <= 0.8) ? sin_rn_small(x) : sin(x);
}
OSG_HD inline double cos_ref(double x)
{
    OSGX_NOCONTRACT
    return (x >= 0.0 && x <= 0.8) ? cos_rn_small(x) : cos(x);
}

}  // namespace osgx
