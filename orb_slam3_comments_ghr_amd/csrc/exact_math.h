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

// ------------------------------------------------------------------ the KannalaBrandt8 projection
// KannalaBrandt8::project / projectJac (ref:src/CameraModels/KannalaBrandt8.cpp:62-80, 229-260) call
// the host libm's double cos(psi), sin(psi) (psi = atan2f(y, x), a float in [-pi, pi]) and
// atan2(r, z).  glibc 2.35 picks an FMA-compiled variant of these at run time on FMA hosts and is not
// correctly rounded: over every 97th float psi in (0, pi], 0.009 % of sin and 0.005 % of cos
// results, and 0.17 % of KB8-range atan2 results, are one ulp off the correctly rounded value
// (tools/glibc_math_check.cc).  As for SE3 exp above, device and oracle therefore both evaluate the
// correctly rounded value, here in double-double with one final rounding, in the oracle via
// __float128 (sinq / cosq / atan2q).  The float atan2f itself is glibc's algorithm, restated bit for
// bit (glibc_math.h).  sincos_psi equals sinq / cosq rounded to double for every float in
// [-pi_f, pi_f] (2.16e9 values, exhaustive: tools/glibc_math_check.cc sincos_psi); atan2_rn equals
// atan2q rounded on 2e8 KB8-range pairs.

OSG_HD inline dd dd_neg(dd a) { return {-a.h, -a.l}; }
OSG_HD inline dd dd_div(dd a, dd b)
{
    OSGX_NOCONTRACT
    const double q1 = a.h / b.h;
    dd r = dd_add(a, dd_neg(dd_mul(b, dd{q1, 0.0})));
    const double q2 = r.h / b.h;
    r = dd_add(r, dd_neg(dd_mul(b, dd{q2, 0.0})));
    const double q3 = r.h / b.h;
    dd q = quick_two_sum(q1, q2);
    return dd_add(q, dd{q3, 0.0});
}

// sin(r), cos(r) of a double-double |r| <= pi/4 + 1e-9: the 15-term series of sin_rn_small /
// cos_rn_small over r^2 in double-double (terms beyond series_terms(|r|) dropped, as there)
OSG_HD inline void sincos_dd_kernel(dd r, dd &s, dd &c)
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
    const dd x2 = dd_mul(r, r);
    const int K = series_terms(fabs(r.h));
    dd a = cs_[14], b = cc_[14];
#pragma unroll
    for (int k = 13; k >= 0; k--) {
        if (k == K - 1) {
            a = cs_[k];
            b = cc_[k];
        } else if (k < K - 1) {
            a = dd_add(dd_mul(a, x2), cs_[k]);
            b = dd_add(dd_mul(b, x2), cc_[k]);
        }
    }
    s = dd_mul(a, r);
    c = b;
}

// sin(x), cos(x) correctly rounded for |x| <= 3.2 (psi of the KB8 projection).  x - n pi/2 with
// n = rint(x 2/pi) in {-2..2}: x - n P1 is exact (n P1 is exact and within a factor of two of x),
// P2 and P3 (pi/2 = P1 + P2 + P3 to 2^-160) are subtracted in double-double.
// Out of line: the callers' other paths (pinhole edges) keep their register budget.
OSG_HD inline __attribute__((noinline)) void sincos_psi(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
    if (x == 0.0) {  // sin(-0) = -0
        sn = x;
        cs = 1.0;
        return;
    }
    const double n = rint(x * 0x1.45f306dc9c883p-1);
    dd r{x, 0.0};
    if (n != 0.0) {
        r = two_sum(x - n * P1, -(n * P2));
        r.l -= n * P3;
        r = quick_two_sum(r.h, r.l);
    }
    dd s, c;
    sincos_dd_kernel(r, s, c);
    const double s1 = s.h + s.l, c1 = c.h + c.l;
    switch (((int)n) & 3) {
    case 0: sn = s1; cs = c1; break;
    case 1: sn = c1; cs = -s1; break;
    case 2: sn = -s1; cs = -c1; break;
    default: sn = -c1; cs = s1; break;
    }
}

// atan2(y, x) correctly rounded (finite, nonzero x and y; the rest is the library's, whose results
// there are exact constants): t = min / max of |x|, |y| in double-double, atan(t) = atan(k / 16) +
// atan(u) with u = (t - k / 16) / (1 + t k / 16), |u| <= 1/32, a 12-term series; then the octant.
OSG_HD inline __attribute__((noinline)) double atan2_rn(double y, double x)
{
    OSGX_NOCONTRACT
    const double ay = fabs(y), ax = fabs(x);
    if (!(ay > 0.0 && ay < INFINITY && ax > 0.0 && ax < INFINITY)) return atan2(y, x);
    const dd tab[17] = {{0.0, 0.0},
                        {0.06241880999595735, -1.5490756308295046e-18},
                        {0.12435499454676144, -3.1253241424539383e-18},
                        {0.18534794999569476, 4.180692268843079e-18},
                        {0.24497866312686414, 1.0698755618734451e-17},
                        {0.3028848683749714, -1.1010827903001369e-17},
                        {0.35877067027057225, -2.4623815582638635e-17},
                        {0.4124104415973873, -1.587652227770689e-17},
                        {0.4636476090008061, 2.2698777452961687e-17},
                        {0.5123894603107377, -2.5462781472855804e-17},
                        {0.5585993153435624, -5.4556305485916264e-18},
                        {0.6022873461349642, 2.950430737228402e-17},
                        {0.6435011087932844, 1.5834785051444286e-17},
                        {0.6823165548747481, 6.943223671560008e-18},
                        {0.7188299996216245, -2.1478388444456983e-17},
                        {0.7531512809621944, -2.4256934659182068e-17},
                        {0.7853981633974483, 3.061616997868383e-17}};
    const dd ser[12] = {{1.0, 0.0},
                        {-0.3333333333333333, -1.850371707708594e-17},
                        {0.2, -1.1102230246251566e-17},
                        {-0.14285714285714285, -7.93016446160826e-18},
                        {0.1111111111111111, 6.1679056923619804e-18},
                        {-0.09090909090909091, 2.523234146875356e-18},
                        {0.07692307692307693, -4.270088556250602e-18},
                        {-0.06666666666666667, -9.251858538542971e-19},
                        {0.058823529411764705, 8.163404592832033e-19},
                        {-0.05263157894736842, -2.921639538487254e-18},
                        {0.047619047619047616, 2.64338815386942e-18},
                        {-0.043478260869565216, -1.206764157201257e-18}};
    const bool swap = ay > ax;
    const double num = swap ? ax : ay, den = swap ? ay : ax;
    const double q1 = num / den;
    const double q2 = fma(-q1, den, num) / den;  // the remainder num - q1 den is exact
    const dd t = quick_two_sum(q1, q2);
    const double k = rint(t.h * 16.0);
    const double ck = k * 0.0625;
    const dd u = dd_div(dd_add(t, dd{-ck, 0.0}), dd_add(dd{1.0, 0.0}, dd_mul(t, dd{ck, 0.0})));
    const dd u2 = dd_mul(u, u);
    dd a = ser[11];
#pragma unroll
    for (int j = 10; j >= 0; j--) a = dd_add(dd_mul(a, u2), ser[j]);
    dd at = dd_add(tab[(int)k], dd_mul(a, u));
    if (swap) at = dd_add(dd{1.5707963267948966, 6.123233995736766e-17}, dd_neg(at));
    if (x < 0.0) at = dd_add(dd{3.141592653589793, 1.2246467991473532e-16}, dd_neg(at));
    const double res = at.h + at.l;
    return y < 0.0 ? -res : res;
}

}  // namespace osgx
