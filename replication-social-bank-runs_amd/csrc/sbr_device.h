// sbr_device.h — device-side building blocks shared by the gfx950 kernels:
// the Tsit5 tableau, OrdinaryDiffEq's PI controller, and exact knot-grid
// lookups (searchsortedlast + Interpolations.jl gridded-linear evaluation).
//
// Every formula here is written to reproduce oracle/sbr_oracle.c bit for bit
// (both sides compile with -ffp-contract=off; fma() only where the oracle has
// it).  The lookups are *faster* than the oracle's — bracketed and galloping
// searches instead of full binary searches — but always return the same
// bracket index, so the interpolated value is identical.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sbr_detmath.h"
#include "../../include/sbr_status.h"

// ode_determine_initdt's exponent 1/(order + 1) with Tsit5's order 5; -DSBR_INITDT_DEN=5 builds
// the alternative the restatement rejected (tools/initdt_evidence.py)
#ifndef SBR_INITDT_DEN
#define SBR_INITDT_DEN 6.0
#endif

namespace sbr {

// ---- Tsit5 (Tsitouras 2011) as in OrdinaryDiffEqTsit5 --------------------
constexpr double C1 = 0.161, C2 = 0.327, C3 = 0.9, C4 = 0.9800255409045097;
constexpr double A21 = 0.161;
constexpr double A31 = -0.008480655492356989, A32 = 0.335480655492357;
constexpr double A41 = 2.897153057105493, A42 = -6.359448489975075, A43 = 4.3622954328695815;
constexpr double A51 = 5.325864828439257, A52 = -11.748883564062828, A53 = 7.4955393428898365,
                 A54 = -0.09249506636175525;
constexpr double A61 = 5.86145544294642, A62 = -12.92096931784711, A63 = 8.159367898576159,
                 A64 = -0.071584973281401, A65 = -0.028269050394068383;
constexpr double A71 = 0.09646076681806523, A72 = 0.01, A73 = 0.4798896504144996, A74 = 1.379008574103742,
                 A75 = -3.290069515436081, A76 = 2.324710524099774;
constexpr double BT1 = -0.00178001105222577714, BT2 = -0.0008164344596567469, BT3 = 0.007880878010261995,
                 BT4 = -0.1447110071732629, BT5 = 0.5823571654525552, BT6 = -0.45808210592918697,
                 BT7 = 0.015151515151515152;
constexpr double TSIT5_STABILITY = 3.5068; // alg_stability_size(::Tsit5)

// ---- PI controller defaults (OrdinaryDiffEqCore, 5th-order method) -------
constexpr double CTL_BETA1 = 0.14, CTL_BETA2 = 0.08, CTL_INV_QMIN = 5.0, CTL_INV_QMAX = 0.1, CTL_GAMMA = 0.9,
                 CTL_QOLDMIN = 1e-4;
constexpr double AUTOSWITCH_TOL = 0.9;
constexpr int AUTOSWITCH_MAXSTIFF = 10, AUTOSWITCH_MAXNONSTIFF = 3;
constexpr double DBL_EPS = 2.220446049250313e-16;

// The bisection's collapse test `abs(d) < 2·eps(d)` (solver.jl:440) in one
// compare: for a normal d, 2·eps(d) = 2^(e-51) is far below |d| ≥ 2^e; for a
// subnormal d, eps(d) = 2^-1074, so the test holds exactly when |d| ≤ 2^-1074
// (d = ±0 or ±denorm_min); NaN and ±Inf fail both forms.
__device__ __forceinline__ bool collapsed(double d) { return fabs(d) <= 4.9406564584124654e-324; }

__device__ __forceinline__ double dmin(double a, double b) { return a < b ? a : b; }
__device__ __forceinline__ double dmax(double a, double b) { return a > b ? a : b; }
// One v_min_f64 / v_max_f64 (IEEE minNum / maxNum) instead of a compare and two
// selects: the same value as dmin / dmax whenever neither operand is NaN and they
// are not zeros of opposite sign — the ODE step-size clamps, whose operands (dt, the
// controller's q) are positive and finite on every step that is kept.
__device__ __forceinline__ double vmin(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ double vmax(double a, double b) { return __builtin_fmax(a, b); }

// a / b for a fixed b by the same IEEE-754 division sequence the compiler
// emits for `/` (v_div_scale, v_rcp_f64, two Newton steps, q = a·r, one fma
// remainder correction, v_div_fmas, v_div_fixup), with the reciprocal refined
// once per constructor instead of per call (3 dependent operations instead of
// ≈11).  Valid where the scale / fixup steps are identities: finite a with
// 2^-969 < |a| < 2^767 (or a = 0, NaN) and a moderate b — there the result is
// the correctly rounded a / b, bit for bit; a = +Inf is selected explicitly.
// Callers: the PI controller's q/γ (q ∈ [1e-45, 1e42]) and the AutoSwitch
// stiffness ratio (only compared with 0.9).
__device__ __forceinline__ double rcp_refined(double b)
{
    double y = __builtin_amdgcn_rcp(b);
    double e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    e = fma(-b, y, 1.0);
    return fma(y, e, y);
}

// a / b given r = rcp_refined(b): the sequence's last three steps.  Bit-identical to
// `a / b` when b is in [2^-960, 2^900] and a is 0 or in [2^-960, 2^767] (no scaling).
__device__ __forceinline__ double div_rcp(double a, double b, double r)
{
    const double q0 = a * r;
    const double rem = fma(-b, q0, a);
    return fma(rem, r, q0);
}

struct ConstDiv {
    double b, r;
    __device__ __forceinline__ explicit ConstDiv(double b_) : b(b_), r(rcp_refined(b_)) {}
    __device__ __forceinline__ double operator()(double a) const
    {
        const double q = div_rcp(a, b, r);
        return a == (double)INFINITY ? (double)INFINITY : q;
    }
    // a known finite (the +Inf select dropped)
    __device__ __forceinline__ double finite(double a) const { return div_rcp(a, b, r); }
};

// AutoSwitch (OrdinaryDiffEqCore composite_algs: maxstiffstep 10, maxnonstiffstep 3,
// stifftol = nonstifftol = 9/10, dtfac 2): in every loopheader!, is_stiff =
// |eigen_est·dt / stability(Tsit5)| > 9/10; successive positives count up, negatives
// down; > 10 switches Tsit5 → Rosenbrock23 (dt ×2), < −3 switches back (dt ÷2).
// choose() returns true when the algorithm changes.
struct AutoSwitch {
    int count = 0;
    int stiff = 0; // 0 / 1 (an int: loop-carried bools cost mask conversions every step)
    int nswitch = 0;
    // |eigen_est·dt / 3.5068| > 9/10 without the division: x ↦ fl(x / 3.5068) is monotone,
    // so the test is |fl(eigen_est·dt)| >= STIFF_THRESHOLD, the least double passing it
    // (tools/stiff_threshold.py; NaN fails both forms)
    static constexpr double STIFF_THRESHOLD = 0x1.93fbbd7b2031ep+1;
    // branch-free (select / toggle): the lanes of a wave switch at different steps
    __device__ __forceinline__ bool choose(double eig, double& dt)
    {
        const bool st = fabs(eig * dt) >= STIFF_THRESHOLD;
        const int cs = count < 0 ? 1 : count + 1, cn = count > 0 ? -1 : count - 1;
        count = st ? cs : cn;
        const bool up = (stiff == 0) & (count > AUTOSWITCH_MAXSTIFF);
        const bool down = (stiff != 0) & (count < -AUTOSWITCH_MAXNONSTIFF);
        const double dt2 = dt * 2.0, dth = dt * 0.5; // dt·0.5 == dt/2 exactly
        dt = down ? dth : dt;
        dt = up ? dt2 : dt;
        stiff ^= (up | down) ? 1 : 0;
        nswitch += (up | down) ? 1 : 0;
        return up | down;
    }
};

// ---- knot-grid lookups ----------------------------------------------------
// searchsortedlast restricted to [lo, hi]; requires t[lo] <= x and that the
// true answer is <= hi.  Returns the largest j in [lo, hi] with t[j] <= x.
template <class P>
__device__ __forceinline__ int ssl_range(P t, int lo, int hi, double x)
{
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (t[mid] <= x) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// searchsortedlast from a hint j0 with t[j0] <= x (exponential gallop forward).
template <class P>
__device__ __forceinline__ int ssl_gallop(P t, int n, int j0, double x)
{
    int lo = j0, step = 1;
    while (lo + step < n && t[lo + step] <= x) {
        lo += step;
        step <<= 1;
    }
    int hi = lo + step - 1;
    if (hi > n - 1) hi = n - 1;
    return ssl_range(t, lo, hi, x);
}

// searchsortedlast from an arbitrary hint h (a prediction, either side of the
// answer): gallop forward or backward from h.  Requires t[0] <= x.
template <class P>
__device__ __forceinline__ int ssl_near(P t, int n, int h, double x)
{
    h = h < 0 ? 0 : (h > n - 1 ? n - 1 : h);
    if (t[h] <= x) return ssl_gallop(t, n, h, x);
    int hi = h - 1, lo = h - 1, step = 1; // invariant: t[hi + 1] > x
    while (lo > 0 && t[lo] > x) {
        hi = lo - 1;
        lo = hi - step;
        step <<= 1;
        if (lo < 0) lo = 0;
    }
    return ssl_range(t, lo, hi, x);
}

// Interpolations.jl gridded Linear on bracket j (clamped to [0, n-2]):
// v[j]*(1-δ) + v[j+1]*δ with δ = (x - t[j]) / (t[j+1] - t[j]).
template <class P, class Q>
__device__ __forceinline__ double lerp_at(P t, Q v, int n, int j, double x)
{
    if (j > n - 2) j = n - 2;
    if (j < 0) j = 0;
    double d = (x - t[j]) / (t[j + 1] - t[j]);
    return v[j] * (1.0 - d) + v[j + 1] * d;
}

}  // namespace sbr
