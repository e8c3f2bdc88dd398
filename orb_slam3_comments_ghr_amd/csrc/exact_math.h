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
// interleaved (the same operations on the same values, so the same two results), which lets a
// latency-bound caller (SE3 exp in the LM loops) overlap them.  The chains enter at term K - 1
// through one switch and run straight on (one branch per call instead of two per unrolled term).
// UNI: every lane holds the same x (PoseOptimization's redundant update), so K is read from the
// first lane and the switch is a scalar branch.
template <bool UNI = false>
OSG_HD inline void sincos_rn_small(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    constexpr dd S0 = {1.0, 0.0}, S1 = {-0.16666666666666666, -9.25185853854297e-18},
                 S2 = {0.008333333333333333, 1.1564823173178714e-19}, S3 = {-0.0001984126984126984, -1.7209558293420705e-22},
                 S4 = {2.7557319223985893e-06, -1.858393274046472e-22}, S5 = {-2.505210838544172e-08, 1.448814070935912e-24},
                 S6 = {1.6059043836821613e-10, 1.2585294588752098e-26}, S7 = {-7.647163731819816e-13, -7.03872877733453e-30},
                 S8 = {2.8114572543455206e-15, 1.6508842730861433e-31}, S9 = {-8.22063524662433e-18, -2.2141894119604265e-34},
                 S10 = {1.9572941063391263e-20, -1.3643503830087908e-36}, S11 = {-3.868170170630684e-23, 8.843177655482344e-40},
                 S12 = {6.446950284384474e-26, -1.9330404233703465e-42}, S13 = {-9.183689863795546e-29, -1.4303150396787322e-45},
                 S14 = {1.1309962886447716e-31, 1.0498015412959506e-47};
    constexpr dd C0 = {1.0, 0.0}, C1 = {-0.5, 0.0}, C2 = {0.041666666666666664, 2.3129646346357427e-18},
                 C3 = {-0.001388888888888889, 5.300543954373577e-20}, C4 = {2.48015873015873e-05, 2.1511947866775882e-23},
                 C5 = {-2.755731922398589e-07, -2.3767714622250297e-23}, C6 = {2.08767569878681e-09, -1.20734505911326e-25},
                 C7 = {-1.1470745597729725e-11, -2.0655512752830745e-28}, C8 = {4.779477332387385e-14, 4.399205485834081e-31},
                 C9 = {-1.5619206968586225e-16, -1.1910679660273754e-32}, C10 = {4.110317623312165e-19, 1.4412973378659527e-36},
                 C11 = {-8.896791392450574e-22, 7.911402614872376e-38}, C12 = {1.6117375710961184e-24, -3.6846573564509766e-41},
                 C13 = {-2.4795962632247976e-27, 1.2953730964765229e-43}, C14 = {3.279889237069838e-30, 1.5117542744029879e-46};
    const dd x2 = two_prod(x, x);
    int K = series_terms(x);
#if defined(__HIP_DEVICE_COMPILE__)
    if (UNI) K = __builtin_amdgcn_readfirstlane(K);
#endif
    dd a, c;
#define OSGX_STEP(k) \
    a = dd_add(dd_mul(a, x2), S##k); \
    c = dd_add(dd_mul(c, x2), C##k)
    switch (K) {
    case 15: a = S14; c = C14; goto t13;
    case 14: a = S13; c = C13; goto t12;
    case 13: a = S12; c = C12; goto t11;
    case 12: a = S11; c = C11; goto t10;
    case 11: a = S10; c = C10; goto t9;
    case 10: a = S9; c = C9; goto t8;
    case 9: a = S8; c = C8; goto t7;
    case 8: a = S7; c = C7; goto t6;
    case 7: a = S6; c = C6; goto t5;
    case 6: a = S5; c = C5; goto t4;
    case 5: a = S4; c = C4; goto t3;
    case 4: a = S3; c = C3; goto t2;
    case 3: a = S2; c = C2; goto t1;
    case 2: a = S1; c = C1; goto t0;
    default: a = S0; c = C0; goto done;
    }
t13: OSGX_STEP(13);
t12: OSGX_STEP(12);
t11: OSGX_STEP(11);
t10: OSGX_STEP(10);
t9: OSGX_STEP(9);
t8: OSGX_STEP(8);
t7: OSGX_STEP(7);
t6: OSGX_STEP(6);
t5: OSGX_STEP(5);
t4: OSGX_STEP(4);
t3: OSGX_STEP(3);
t2: OSGX_STEP(2);
t1: OSGX_STEP(1);
t0: OSGX_STEP(0);
done:
#undef OSGX_STEP
    const dd r = dd_mul(a, dd{x, 0.0});
    sn = r.h + r.l;
    cs = c.h + c.l;
}
template <bool UNI = false>
OSG_HD inline void sincos_ref(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    if (x >= 0.0 && x <= 0.8) {
        sincos_rn_small<UNI>(x, sn, cs);
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
// a + b without the second two_sum of dd_add ("sloppy" addition): ~2^-104 relative error unless
// a and b nearly cancel, which none of the uses below does
OSG_HD inline dd dd_add_s(dd a, dd b)
{
    OSGX_NOCONTRACT
    dd s = two_sum(a.h, b.h);
    s.l += a.l + b.l;
    return quick_two_sum(s.h, s.l);
}
// a + b for a double b
OSG_HD inline dd dd_add_d(dd a, double b)
{
    OSGX_NOCONTRACT
    dd s = two_sum(a.h, b);
    s.l += a.l;
    return quick_two_sum(s.h, s.l);
}
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

// sin / cos (k / 32), k = 0..25, as double-double pairs {sin.h, sin.l, cos.h, cos.l}
#define OSGX_SINCOS32_TABLE \
        {0.0, 0.0, 1.0, 0.0}, \
        {0.03124491398532608, -1.562781562225433e-18, 0.9995117584851364, -3.418806487972947e-17}, \
        {0.0624593178423802, -2.040259504585711e-18, 0.9980475107000991, 3.3232291674141346e-17}, \
        {0.09361273123551289, 1.4628632005878733e-18, 0.9956086864580017, 3.312922430932991e-17}, \
        {0.12467473338522769, -2.925947496057858e-18, 0.992197667229329, 4.754870575189364e-17}, \
        {0.15561499277355603, 8.886053372342288e-18, 0.9878177838164719, 4.91917302237681e-17}, \
        {0.18640329676226988, 2.3493796901281573e-18, 0.9824733131012553, -3.919920375420088e-17}, \
        {0.21700958109501015, 1.1170071073364376e-17, 0.9761694738686353, -7.850690609285027e-18}, \
        {0.24740395925452294, -7.53102495590706e-18, 0.9689124217106447, 5.071436662403936e-17}, \
        {0.2775567516463363, 1.7674070262791822e-17, 0.9607092430155619, -2.807827063516729e-17}, \
        {0.30743851458038085, 1.1004366442765296e-19, 0.9515679480481722, -3.8614834675674123e-17}, \
        {0.33702006902225307, 1.0312279860787216e-17, 0.9414974631278811, -4.8523830236797095e-18}, \
        {0.36627252908604757, -9.938814562106524e-18, 0.9305076219123143, 4.488760003328074e-18}, \
        {0.39516733024093426, -1.9613487871414228e-17, 0.9186091557949183, -4.0564150104514996e-17}, \
        {0.42367625720393803, -2.331800700068871e-17, 0.9058136834259364, 4.2864666490805214e-17}, \
        {0.4517714714916838, -8.234073942098903e-18, 0.8921336993669944, 2.3160655211380166e-17}, \
        {0.479425538604203, -5.103969860556013e-18, 0.8775825618903728, -4.2623149864279997e-17}, \
        {0.5066114548142574, -3.269413423618168e-17, 0.8621744799348805, 4.4132427578105805e-18}, \
        {0.5333026735360201, 5.129318115032044e-17, 0.8459244992310679, 1.549506647350329e-17}, \
        {0.5594731312473669, 1.575565514488728e-17, 0.8288484876093257, 1.1163935406617444e-17}, \
        {0.5850972729404622, -5.4883972461161805e-17, 0.8109631195052179, -3.091333486122179e-17}, \
        {0.6101500770757914, -1.479826990758988e-17, 0.7922858596771786, -2.9049779312834576e-17}, \
        {0.6346070800152693, -3.4568582392624965e-17, 0.7728349461524715, 4.231014921891023e-17}, \
        {0.6584443999105676, -3.7736386700306717e-17, 0.7526293724180665, -1.2970993013150526e-17}, \
        {0.6816387600233341, 4.410467313197903e-17, 0.7316888688738209, -1.0475824306512768e-17}, \
        {0.7041675114545337, -3.94095700584825e-17, 0.7100338835660797, 1.505272211891291e-17}
// atan(k / 64), k = 0..64, double-double
#define OSGX_ATAN64_TABLE \
        {0.0, 0.0}, \
        {0.015623728620476831, -4.913600136566304e-19}, \
        {0.031239833430268277, -1.188442711587748e-18}, \
        {0.046840712915969654, -1.655677442254952e-19}, \
        {0.06241880999595735, -1.5490756308295046e-18}, \
        {0.0779666338315423, 5.804551873143357e-18}, \
        {0.09347678115858947, -6.2844725995420954e-18}, \
        {0.10894195698986579, 6.8267122072409585e-18}, \
        {0.12435499454676144, -3.1253241424539383e-18}, \
        {0.13970887428916365, -2.9579864247315813e-18}, \
        {0.15499674192394097, 9.585415594114324e-18}, \
        {0.1702119252854744, -3.541164079802125e-18}, \
        {0.18534794999569476, 4.180692268843079e-18}, \
        {0.2003985538258785, 3.1399542871844493e-18}, \
        {0.21535769969773805, 4.738160130078733e-19}, \
        {0.23021958727684372, 1.2313404529142703e-17}, \
        {0.24497866312686414, 1.0698755618734451e-17}, \
        {0.2596296294082575, 1.9238754924615304e-17}, \
        {0.2741674511196588, 8.261353575163773e-18}, \
        {0.2885873618940774, -1.428369957377257e-17}, \
        {0.3028848683749714, -1.1010827903001369e-17}, \
        {0.31705575320914703, -1.893928924292642e-17}, \
        {0.3310960767041321, -7.952610375793799e-18}, \
        {0.34500217720710513, -2.2938804755578304e-17}, \
        {0.35877067027057225, -2.4623815582638635e-17}, \
        {0.3723984466767542, 1.9612311504845653e-17}, \
        {0.38588266939807375, 2.378822732491941e-17}, \
        {0.39922076957525254, 2.246598105617042e-17}, \
        {0.4124104415973873, -1.587652227770689e-17}, \
        {0.42544963737004227, 2.3315530741892885e-17}, \
        {0.43833655985795783, -2.494277030626541e-17}, \
        {0.4510696559885235, -2.2703795229420475e-17}, \
        {0.4636476090008061, 2.2698777452961687e-17}, \
        {0.4760693303227612, 1.4654487332256713e-17}, \
        {0.48833395105640554, -1.1373236189329585e-17}, \
        {0.5004408131472942, -4.7181675085518756e-17}, \
        {0.5123894603107377, -2.5462781472855804e-17}, \
        {0.5241796287829132, 5.520094119641666e-18}, \
        {0.5358112379604637, -4.0637956834825575e-18}, \
        {0.5472843809874369, 4.923709671396255e-17}, \
        {0.5585993153435624, -5.4556305485916264e-18}, \
        {0.5697564534829784, 1.2255062085054184e-17}, \
        {0.5807563535676704, -1.441464378193067e-17}, \
        {0.5915997103351114, 4.920495453686772e-17}, \
        {0.6022873461349642, 2.950430737228402e-17}, \
        {0.6128202021652414, -3.1552061848586226e-17}, \
        {0.6231993299340659, 2.672403885140095e-17}, \
        {0.6334258829691446, -2.7290767436015276e-17}, \
        {0.6435011087932844, 1.5834785051444286e-17}, \
        {0.6534263411807619, 3.5800634857340095e-17}, \
        {0.6632029927060933, -3.076054864429649e-17}, \
        {0.6728325475937632, -1.899315009714705e-17}, \
        {0.6823165548747481, 6.943223671560008e-18}, \
        {0.6916566218531999, -8.117151192285796e-18}, \
        {0.7008544078844502, -1.987626234335816e-17}, \
        {0.7099116184635249, -4.597166450584887e-17}, \
        {0.7188299996216245, -2.1478388444456983e-17}, \
        {0.7276113326265107, 2.569325697391839e-18}, \
        {0.7362574289814281, 3.473937648299457e-17}, \
        {0.7447701257160751, 3.708315849135547e-17}, \
        {0.7531512809621944, -2.4256934659182068e-17}, \
        {0.7614027698055784, 9.850030332752822e-18}, \
        {0.7695264804056583, -3.704991905602721e-17}, \
        {0.7775243103733478, -2.6676490951944502e-17}, \
        {0.7853981633974483, 3.061616997868383e-17}

// sin(x), cos(x) correctly rounded for |x| <= 3.2 (psi of the KB8 projection).
//   * x - n pi/2 with n = rint(x 2/pi) in {-2..2}: x - n P1 is exact (n P1 is exact and within a
//     factor of two of x), P2 and P3 (pi/2 = P1 + P2 + P3 to 2^-160) are subtracted in double-double;
//   * r = a + t with a = k / 32 (table) and |t| <= 1/64 (t = r - a exact by Sterbenz for k != 0);
//   * sin t = t + t^3 (-1/6 + t^2 q_s), cos t = 1 + t^2 (-1/2 + t^2 q_c): the leading coefficients
//     in double-double, the short tails q_s, q_c (|t^2 q| < 2^-20) in double, so the whole value
//     carries ~2^-100 relative error; sin r = S cos t + C sin t, cos r = C cos t - S sin t.
// One final rounding.  Out of line: the callers' other paths (pinhole edges) keep their register
// budget.
OSG_HD inline __attribute__((noinline)) void sincos_psi(double x, double &sn, double &cs)
{
    OSGX_NOCONTRACT
    if (x == 0.0) {  // sin(-0) = -0
        sn = x;
        cs = 1.0;
        return;
    }
    const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
    const double n = rint(x * 0x1.45f306dc9c883p-1);
    dd r{x, 0.0};
    if (n != 0.0) {
        r = two_sum(x - n * P1, -(n * P2));
        r.l -= n * P3;
        r = quick_two_sum(r.h, r.l);
    }
    static const double tab[26][4] = {OSGX_SINCOS32_TABLE};
    const double kf = rint(r.h * 32.0);
    const int ak = (int)fabs(kf);
    const dd t = two_sum(r.h - kf * 0.03125, r.l);
    const dd t2 = dd_mul(t, t);
    const double z = t2.h;
    const double qs = z * (1.0 / 120.0 + z * (-1.0 / 5040.0 + z * (1.0 / 362880.0)));
    const double qc = z * (1.0 / 24.0 + z * (-1.0 / 720.0 + z * (1.0 / 40320.0)));
    const dd sin_t = dd_add_s(t, dd_mul(dd_mul(t, t2), dd_add_d(dd{-0.16666666666666666, -9.25185853854297e-18}, qs)));
    const dd cos_t = dd_add_d(dd_mul(t2, dd_add_d(dd{-0.5, 0.0}, qc)), 1.0);
    const double sg = kf < 0.0 ? -1.0 : 1.0;
    const dd S{sg * tab[ak][0], sg * tab[ak][1]}, C{tab[ak][2], tab[ak][3]};
    const dd sr = dd_add_s(dd_mul(S, cos_t), dd_mul(C, sin_t));
    const dd cr = dd_add_s(dd_mul(C, cos_t), dd_neg(dd_mul(S, sin_t)));
    const double s1 = sr.h + sr.l, c1 = cr.h + cr.l;
    switch (((int)n) & 3) {
    case 0: sn = s1; cs = c1; break;
    case 1: sn = c1; cs = -s1; break;
    case 2: sn = -s1; cs = -c1; break;
    default: sn = -c1; cs = s1; break;
    }
}

// atan2(y, x) correctly rounded (finite, nonzero x and y; the rest is the library's, whose results
// there are exact constants): t = min / max of |x|, |y| in double-double, atan(t) = atan(k / 64) +
// atan(u) with u = (t - k / 64) / (1 + t k / 64), |u| <= 1/128, atan u = u + u^3 (-1/3 + u^2 q)
// (the tail q in double, |u^2 q| < 2^-14); then the octant.  ~2^-100 relative error, one rounding.
OSG_HD inline __attribute__((noinline)) double atan2_rn(double y, double x)
{
    OSGX_NOCONTRACT
    const double ay = fabs(y), ax = fabs(x);
    if (!(ay > 0.0 && ay < INFINITY && ax > 0.0 && ax < INFINITY)) return atan2(y, x);
    static const double tab[65][2] = {OSGX_ATAN64_TABLE};
    const bool swap = ay > ax;
    const double num = swap ? ax : ay, den = swap ? ay : ax;
    const double q1 = num / den;
    const double q2 = fma(-q1, den, num) / den;  // the remainder num - q1 den is exact
    const dd t = quick_two_sum(q1, q2);
    const double k = rint(t.h * 64.0);
    const double ck = k * 0.015625;
    const dd u = dd_div(dd_add_d(t, -ck), dd_add_d(dd_mul(t, dd{ck, 0.0}), 1.0));
    const dd u2 = dd_mul(u, u);
    const double z = u2.h;
    const double q = z * (0.2 + z * (-1.0 / 7.0 + z * (1.0 / 9.0 + z * (-1.0 / 11.0))));
    const dd au = dd_add_s(u, dd_mul(dd_mul(u, u2), dd_add_d(dd{-0.3333333333333333, -1.850371707708594e-17}, q)));
    const int ik = (int)k;
    dd at = dd_add_s(dd{tab[ik][0], tab[ik][1]}, au);
    if (swap) at = dd_add_s(dd{1.5707963267948966, 6.123233995736766e-17}, dd_neg(at));
    if (x < 0.0) at = dd_add_s(dd{3.141592653589793, 1.2246467991473532e-16}, dd_neg(at));
    const double res = at.h + at.l;
    return y < 0.0 ? -res : res;
}

}  // namespace osgx
