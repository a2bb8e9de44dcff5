/*
 * sbr_detmath.h — deterministic FP64 elementary functions shared by the HIP
 * kernels and the CPU oracle.
 *
 * Why this exists: the reference (Julia) evaluates exp() in the hazard rate
 * (src/baseline/solver.jl:168,181) and x^y in the step-size controller and
 * the initial-dt heuristic of OrdinaryDiffEq (not vendored; see SURVEY.md
 * §8(a) a15).  The GPU's ocml exp/log and glibc's exp/log are both < 1 ulp
 * but not bit-identical, which would make GPU-vs-oracle parity a tolerance
 * question and let run/no-run decisions flip at boundaries.  Both sides
 * therefore call these functions: plain IEEE double arithmetic only (+ - * /,
 * no fma), evaluated in the written order (every consumer is compiled with
 * -ffp-contract=off), so the host and gfx950 results are bit-identical.
 *
 * Algorithms: the classic Cody–Waite reduced exp with a degree-5 rational
 * remez correction and the atanh-series log (the fdlibm formulation, public
 * domain algorithm).  Accuracy < 1 ulp in the ranges used here.  They are
 * NOT Julia's Base.exp / Base.log bit-for-bit: those are table-driven; the
 * difference is ≤ 1 ulp and is covered by the parity statement in DESIGN.md.
 */
#ifndef SBR_DETMATH_H
#define SBR_DETMATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define SBR_HD __host__ __device__ static inline
#else
#define SBR_HD static inline
#endif

SBR_HD uint64_t sbr_dbits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
SBR_HD double sbr_bitsd(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }

/* 2^k for -1074 <= k <= 1023, built from bits (exact). */
SBR_HD double sbr_pow2i(int k)
{
    if (k >= -1022) return sbr_bitsd((uint64_t)(k + 1023) << 52);
    return sbr_bitsd((uint64_t)1 << (k + 1074)); /* subnormal */
}

/* Julia's eps(x) for Float64 (base/float.jl): ldexp(eps(), exponent(x)) for
 * normal x, nextfloat(0.0) for zero/subnormal, NaN for non-finite. */
SBR_HD double sbr_jl_eps(double x)
{
    uint64_t b = sbr_dbits(x) & 0x7fffffffffffffffull;
    int e = (int)(b >> 52);
    if (e == 0x7ff) return sbr_bitsd(0x7ff8000000000000ull);
    if (e == 0) return sbr_bitsd(1ull); /* 5e-324 */
    return sbr_pow2i(e - 1023 - 52);
}

#define SBR_LN2_HI 6.93147180369123816490e-01
#define SBR_LN2_LO 1.90821492927058770002e-10
#define SBR_INV_LN2 1.44269504088896338700e+00

SBR_HD double sbr_exp(double x)
{
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    if (x != x) return x;
    if (x > 7.09782712893383973096e+02) return sbr_bitsd(0x7ff0000000000000ull);
    if (x < -7.45133219101941108420e+02) return 0.0;
    double t = x * SBR_INV_LN2;
    int k = (int)(t < 0.0 ? t - 0.5 : t + 0.5);
    double kd = (double)k;
    double hi = x - kd * SBR_LN2_HI; /* exact: LN2_HI has 20 trailing zero bits */
    double lo = kd * SBR_LN2_LO;
    double r = hi - lo;
    double r2 = r * r;
    double c = r - r2 * (P1 + r2 * (P2 + r2 * (P3 + r2 * (P4 + r2 * P5))));
    double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    if (k > 1023) return y * 2.0 * sbr_pow2i(k - 1);
    if (k < -1021) return (y * sbr_pow2i(k + 54)) * sbr_pow2i(-54);
    return y * sbr_pow2i(k);
}

SBR_HD double sbr_log(double x)
{
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01;
    const double Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01;
    const double Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01;
    const double Lg7 = 1.479819860511658591e-01;
    if (x != x) return x;
    if (x < 0.0) return sbr_bitsd(0x7ff8000000000000ull);
    if (x == 0.0) return sbr_bitsd(0xfff0000000000000ull);
    uint64_t b = sbr_dbits(x);
    if ((b >> 52) == 0x7ff) return x; /* +inf */
    int k = 0;
    if ((b >> 52) == 0) { x = x * 18014398509481984.0; k = -54; b = sbr_dbits(x); } /* 2^54 */
    uint32_t hx = (uint32_t)(b >> 32);
    k += (int)(hx >> 20) - 1023;
    hx &= 0x000fffffu;
    uint32_t i = (hx + 0x95f64u) & 0x100000u; /* mantissa >= sqrt(2)? then halve */
    b = ((uint64_t)(hx | (i ^ 0x3ff00000u)) << 32) | (b & 0xffffffffull);
    k += (int)(i >> 20);
    double m = sbr_bitsd(b);
    double f = m - 1.0;
    double s = f / (2.0 + f);
    double z = s * s;
    double w = z * z;
    double R = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7))) + w * (Lg2 + w * (Lg4 + w * Lg6));
    double hfsq = 0.5 * f * f;
    double dk = (double)k;
    return dk * SBR_LN2_HI - ((hfsq - (s * (hfsq + R) + dk * SBR_LN2_LO)) - f);
}

/* x^y for x > 0 (controller / initial-dt use only). */
SBR_HD double sbr_pow_pos(double x, double y)
{
    if (x == 0.0) return 0.0;
    return sbr_exp(y * sbr_log(x));
}

#endif /* SBR_DETMATH_H */
