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
 * therefore call these functions: plain IEEE double arithmetic (+ - * / and
 * explicit fma(), which is exact on both sides: v_fma_f64 / vfmadd), evaluated
 * in the written order (every consumer is compiled with -ffp-contract=off),
 * so the host and gfx950 results are bit-identical.
 *
 * Algorithms: the classic Cody–Waite reduced exp with a degree-5 rational
 * remez correction and the atanh-series log (the fdlibm formulations, public
 * domain algorithms; the log polynomial in fma).  Accuracy < 1 ulp in the
 * ranges used here.  (An fma/Estrin exp without the division was tried: its
 * different last-bit rounding moved one column of the 5000² paper mask —
 * tools/check_mask5000.py — so the figure-pinned formulation stays.)  They are
 * NOT Julia's Base.exp / Base.log bit-for-bit: those are table-driven; the
 * difference is ≤ 1 ulp and is covered by the parity statement in DESIGN.md.
 */
#ifndef SBR_DETMATH_H
#define SBR_DETMATH_H

#include <stdint.h>
#if !defined(__HIPCC__)
#include <math.h>
#endif

#if defined(__HIPCC__)
#define SBR_HD __host__ __device__ static inline
#else
#define SBR_HD static inline
#endif

SBR_HD uint64_t sbr_dbits(double x) { uint64_t u; __builtin_memcpy(&u, &x, 8); return u; }
SBR_HD double sbr_bitsd(uint64_t u) { double x; __builtin_memcpy(&x, &u, 8); return x; }

/* 2^k for -1074 <= k <= 1023, built from bits (exact).  Branch-free: both
 * encodings are formed and one is selected (k is clamped so every shift is
 * defined), so a divergent wave runs one straight-line sequence. */
SBR_HD double sbr_pow2i(int k)
{
    const int kn = k < -1022 ? -1022 : (k > 1023 ? 1023 : k);
    const int ks = k < -1074 ? 0 : (k > -1023 ? 0 : k + 1074);
    const uint64_t bn = (uint64_t)(kn + 1023) << 52;
    const uint64_t bs = (uint64_t)1 << ks;
    return sbr_bitsd(k >= -1022 ? bn : bs);
}

/* Julia's eps(x) for Float64 (base/float.jl): ldexp(eps(), exponent(x)) for
 * normal x, nextfloat(0.0) for zero/subnormal, NaN for non-finite. */
SBR_HD double sbr_jl_eps(double x)
{
    const uint64_t b = sbr_dbits(x) & 0x7fffffffffffffffull;
    const int e = (int)(b >> 52);
    const double r = sbr_pow2i(e - 1023 - 52);
    const double tiny = sbr_bitsd(1ull); /* 5e-324 */
    const double qnan = sbr_bitsd(0x7ff8000000000000ull);
    return e == 0x7ff ? qnan : (e == 0 ? tiny : r);
}

#define SBR_LN2_HI 6.93147180369123816490e-01
#define SBR_LN2_LO 1.90821492927058770002e-10
#define SBR_INV_LN2 1.44269504088896338700e+00

/* (r·c) / (2 − c) of sbr_exp, correctly rounded.  On gfx950 for the fast path's operands
 * (a = 0 or 2^-900 < |a| < 1, b in [1.6, 2.4]) the compiler's IEEE division sequence without
 * its v_div_scale / v_div_fmas scaling and v_div_fixup special-case steps, which are identities
 * there (v_rcp_f64, two Newton steps on the reciprocal, q = a·r, one fma remainder correction):
 * the same quotient bit for bit; the host divides. */
SBR_HD double sbr_ddiv_mid(double a, double b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    double y = __builtin_amdgcn_rcp(b);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-b, q, a), y, q);
#else
    return a / b;
#endif
}

/* sbr_exp for x = 0 or 2^-400 <= |x| <= 708 (k in [-1021, 1021]: the normal-result branch,
 * no special input): the same operations as sbr_exp's, so the same bits, without the
 * special-input and sub/overnormal selects. */
SBR_HD double sbr_exp_mid(double x)
{
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    const double t = x * SBR_INV_LN2;
    const int k = (int)(t < 0.0 ? t - 0.5 : t + 0.5);
    const double kd = (double)k;
    const double hi = x - kd * SBR_LN2_HI;
    const double lo = kd * SBR_LN2_LO;
    const double r = hi - lo;
    const double r2 = r * r;
    const double c = r - r2 * (P1 + r2 * (P2 + r2 * (P3 + r2 * (P4 + r2 * P5))));
    const double y = 1.0 - ((lo - sbr_ddiv_mid(r * c, 2.0 - c)) - hi);
    return y * sbr_bitsd((uint64_t)(k + 1023) << 52);
}

/* exp: Cody–Waite reduction x = k ln2 + r, |r| <= ln2/2, then the fdlibm
 * rational form.  Special inputs are computed on a safe argument and
 * replaced by select at the end.  On the device the common range takes
 * sbr_exp_mid (same bits) behind one branch, which a wave whose lanes all
 * hold such arguments never leaves. */
SBR_HD double sbr_exp_full(double x);
SBR_HD double sbr_exp(double x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const double ax = __builtin_fabs(x);
    if ((ax <= 708.0 && ax >= 0x1p-400) || x == 0.0) return sbr_exp_mid(x);
#endif
    return sbr_exp_full(x);
}

SBR_HD double sbr_exp_full(double x)
{
    const double P1 = 1.66666666666666019037e-01;
    const double P2 = -2.77777777770155933842e-03;
    const double P3 = 6.61375632143793436117e-05;
    const double P4 = -1.65339022054652515390e-06;
    const double P5 = 4.13813679705723846039e-08;
    const int isnan_ = x != x;
    const int over = x > 7.09782712893383973096e+02;
    const int under = x < -7.45133219101941108420e+02;
    const double xs = (isnan_ | over | under) ? 0.0 : x;
    const double t = xs * SBR_INV_LN2;
    const int k = (int)(t < 0.0 ? t - 0.5 : t + 0.5); /* |k| <= 1075 */
    const double kd = (double)k;
    const double hi = xs - kd * SBR_LN2_HI; /* exact: LN2_HI has 20 trailing zero bits */
    const double lo = kd * SBR_LN2_LO;
    const double r = hi - lo;
    const double r2 = r * r;
    const double c = r - r2 * (P1 + r2 * (P2 + r2 * (P3 + r2 * (P4 + r2 * P5))));
    const double y = 1.0 - ((lo - (r * c) / (2.0 - c)) - hi);
    const double y_big = y * 2.0 * sbr_pow2i(k - 1);                    /* k == 1024 */
    const double y_sub = (y * sbr_pow2i(k + 54)) * sbr_pow2i(-54);      /* k < -1021 */
    const double y_nrm = y * sbr_pow2i(k);
    const double res = k > 1023 ? y_big : (k < -1021 ? y_sub : y_nrm);
    const double inf = sbr_bitsd(0x7ff0000000000000ull);
    return isnan_ ? x : (over ? inf : (under ? 0.0 : res));
}

/* log: x = 2^k m, m in [sqrt(2)/2, sqrt(2)), log(m) = 2 atanh(f/(2+f)) with
 * the fdlibm polynomial, evaluated in fma.  Branch-free; special inputs
 * selected at the end. */
SBR_HD double sbr_log(double x)
{
    const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01;
    const double Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01;
    const double Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01;
    const double Lg7 = 1.479819860511658591e-01;
    const uint64_t b0 = sbr_dbits(x);
    const int special = (x != x) | (x <= 0.0) | ((b0 >> 52) >= 0x7ff);
    const int sub = ((b0 >> 52) == 0) & !special;
    const double xs = special ? 1.0 : (sub ? x * 18014398509481984.0 : x); /* 2^54 */
    int k = sub ? -54 : 0;
    uint64_t b = sbr_dbits(xs);
    uint32_t hx = (uint32_t)(b >> 32);
    k += (int)(hx >> 20) - 1023;
    hx &= 0x000fffffu;
    const uint32_t i = (hx + 0x95f64u) & 0x100000u; /* mantissa >= sqrt(2)? then halve */
    b = ((uint64_t)(hx | (i ^ 0x3ff00000u)) << 32) | (b & 0xffffffffull);
    k += (int)(i >> 20);
    const double m = sbr_bitsd(b);
    const double f = m - 1.0;
    const double s = f / (2.0 + f);
    const double z = s * s;
    const double w = z * z;
    const double t1 = w * fma(w, fma(w, Lg6, Lg4), Lg2);
    const double t2 = z * fma(w, fma(w, fma(w, Lg7, Lg5), Lg3), Lg1);
    const double R = t2 + t1;
    const double hfsq = (0.5 * f) * f;
    const double dk = (double)k;
    const double res = dk * SBR_LN2_HI - ((hfsq - fma(s, hfsq + R, dk * SBR_LN2_LO)) - f);
    const double qnan = sbr_bitsd(0x7ff8000000000000ull);
    const double ninf = sbr_bitsd(0xfff0000000000000ull);
    const double sp = (x != x) ? x : (x < 0.0 ? qnan : (x == 0.0 ? ninf : x)); /* +inf -> +inf */
    return special ? sp : res;
}

/* x^y for x > 0 (initial-dt use only). */
SBR_HD double sbr_pow_pos(double x, double y)
{
    return x == 0.0 ? 0.0 : sbr_exp(y * sbr_log(x));
}

/* 10^y, log10(x) for the initial-dt heuristic (ode_determine_initdt's
 * 10.0^(-(2 + log10(d)) / order)); Julia's Base log10 / ^ are not restated
 * bit for bit — the first dt is "parity unpinned" at the ulp level. */
#define SBR_LN10 2.30258509299404568402e+00
SBR_HD double sbr_log10(double x) { return sbr_log(x) / SBR_LN10; }
SBR_HD double sbr_exp10(double y) { return sbr_exp(y * SBR_LN10); }

/* ------------------------------------------------------------------------
 * FastPower.fastpower (FastPower 1.1.3, Manifest.toml:675-678; called by
 * OrdinaryDiffEqCore's PIController, stepsize_controller!): a Float32
 * approximation of x^y,
 *     fastpower(x, y) = Float64(@fastmath exp2(Float32(y) * fastlog2(Float32(x))))
 * with fastlog2 the rational approximation (x-1)(a(x-1)+b)/((x-1)+c) of
 * Goldberg's "fast approximate logarithms" (table 2, line 8) on the
 * significand, and Julia's Base.Math exp2 for Float32 (exp_impl_fast:
 * N = round(x), r = x - N, the degree-7 Horner kernel in muladd, times 2^N).
 * Restated from the published algorithm (not vendored).  All Float32
 * arithmetic is IEEE single precision, evaluated as written (callers are
 * compiled with -ffp-contract=off; fmaf only where Julia's evalpoly has a
 * muladd); identical on the host and gfx950.
 * ------------------------------------------------------------------------ */
SBR_HD uint32_t sbr_fbits(float x) { uint32_t u; __builtin_memcpy(&u, &x, 4); return u; }
SBR_HD float sbr_bitsf(uint32_t u) { float x; __builtin_memcpy(&x, &u, 4); return x; }

/* n / d in IEEE single precision for d in [1, 4) and n = 0 or 2^-100 < |n| < 2^100: on
 * gfx950 the hardware division sequence the compiler emits for `/` (v_rcp_f32, one
 * Newton step on the reciprocal, q = n·r, two fma remainder corrections) without its
 * v_div_scale / v_div_fmas scaling and v_div_fixup special-case steps, which are
 * identities for these operands — the same correctly rounded quotient, bit for bit,
 * in 8 dependent operations instead of 11; the host divides. */
SBR_HD float sbr_fdiv_mid(float n, float d)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const float r0 = __builtin_amdgcn_rcpf(d);
    const float r = __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
    float q = n * r;
    q = __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
    return __builtin_fmaf(__builtin_fmaf(-d, q, n), r, q);
#else
    return n / d;
#endif
}

SBR_HD float sbr_fastlog2f(float x)
{
    const float a = 0.338953f, b = 2.198599f, c = 1.523692f;
    const uint32_t ux1i = sbr_fbits(x);
    const uint32_t e = (ux1i & 0x7F800000u) >> 23;
    const uint32_t g = (ux1i >> 22) & 1u; /* significand > 1.5 */
    /* g: halve the significand (exponent 0x3f000000 instead of 0x3f800000) and
     * compensate with 126 instead of 127 (integer forms of the same selects) */
    const float signif0 = sbr_bitsf(((ux1i & 0x007FFFFFu) | 0x3f800000u) - (g << 23));
    const float fexp = (float)((int32_t)e - 127 + (int32_t)g);
    const float signif = signif0 - 1.0f;
    /* signif in [-0.25, 0.5): the divisor signif + c is in [1.27, 2.03) */
    return fexp + sbr_fdiv_mid(signif * (a * signif + b), signif + c);
}

/* Base.Math.exp_impl_fast(x::Float32, Val(2)) (MAX_EXP = 128, SUBNORM_EXP = 150).
 * Branch-free: the kernel runs on a clamped argument and the out-of-range / NaN
 * results are selected at the end (NaN in -> NaN out, as Julia's NaN * 2^N). */
SBR_HD float sbr_exp2f_jl(float x)
{
    const int over = x >= 128.0f, under = x <= -150.0f, nan_ = x != x;
    /* the kernel's argument clamped into [-150, 128] (NaN -> -150): out-of-range and NaN
     * results are selected at the end, the clamp only keeps the exponent arithmetic defined */
    const float xs = __builtin_fminf(__builtin_fmaxf(x, -150.0f), 128.0f);
    const float nf = __builtin_rintf(xs); /* round(x), ties to even */
    const float r0 = __builtin_fmaf(nf, -1.0f, xs);
    const float r = __builtin_fmaf(nf, 0.0f, r0);
    float p = 1.5316464e-5f; /* expb_kernel(Val(2), ::Float32): evalpoly = Horner in muladd */
    p = __builtin_fmaf(r, p, 0.00015469732f);
    p = __builtin_fmaf(r, p, 0.0013333423f);
    p = __builtin_fmaf(r, p, 0.009618025f);
    p = __builtin_fmaf(r, p, 0.05550411f);
    p = __builtin_fmaf(r, p, 0.2402265f);
    p = __builtin_fmaf(r, p, 0.6931472f);
    p = __builtin_fmaf(r, p, 1.0f);
    const int32_t n = (int32_t)nf;
    const float twopk = sbr_bitsf((uint32_t)(n + 127) << 23);
    const float res = twopk * p;
    /* one select per case on computed values (no conditional arms to branch over) */
    const float inf = sbr_bitsf(0x7f800000u);
    float out = nan_ ? x : res;
    out = under ? 0.0f : out;
    out = over ? inf : out;
    return out;
}

/* FastPower.fastpower(x, y) for Float64 x, y */
SBR_HD double sbr_fastpow(double x, double y)
{
    if (x == 0.0) return 0.0;
    const uint64_t bx = sbr_dbits(x) & 0x7fffffffffffffffull, by = sbr_dbits(y) & 0x7fffffffffffffffull;
    if (bx == 0x7ff0000000000000ull && by == 0x7ff0000000000000ull) return sbr_bitsd(0x7ff0000000000000ull);
    return (double)sbr_exp2f_jl((float)y * sbr_fastlog2f((float)x));
}

#endif /* SBR_DETMATH_H */
