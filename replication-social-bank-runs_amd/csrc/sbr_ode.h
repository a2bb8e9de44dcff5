// sbr_ode.h — OrdinaryDiffEq's AutoTsit5(Rosenbrock23()) at reltol = abstol =
// eps() on the device: one lane integrates one ODE.  The reference solves every
// learning / value-function ODE with it (learning.jl:51,
// heterogeneity_learning.jl:74, social_learning_dynamics.jl:71,
// value_function_solver.jl:105; OrdinaryDiffEqCore 1.34.0, OrdinaryDiffEqTsit5
// 1.5.0, OrdinaryDiffEqRosenbrock 1.18.1 — not vendored, restated in
// oracle/sbr_oracle.c, which these routines match bit for bit):
//
//   * ode_determine_initdt (Tsit5 current at init);
//   * per loop iteration (loopheader!): AutoSwitch's stiffness test on the
//     last eigen_est and the proposed dt — 11 successive positives switch to
//     Rosenbrock23 (dt ×2), 4 successive negatives switch back (dt ÷2); the
//     new algorithm re-evaluates fsalfirst = f(uprev, t);
//   * Tsit5 (eigen_est = |(k7 − k6)/(u − g6)|) or Rosenbrock23 (eigen_est =
//     ‖J‖_∞, W = J − I/(dt·d), three linear solves);
//   * the PI controller with FastPower.fastpower (Float32) for EEst^β1 and
//     qold^β2, accept / reject, tstop clipping and the 100·eps snap.
//
// Scalar systems (baseline learning, social forced ODE, interest value function)
// use ode_scalar; the K-group hetero system has its own loop (sbr_hetero.hip)
// on the same PIControl / AutoSwitch / Rosenbrock23 pieces.
#pragma once

#include <type_traits>
#include <utility>

#include "sbr_device.h"

namespace sbr {

// Rosenbrock23Tableau: c32 = 6 + sqrt(2), d = 1/(2 + sqrt(2))
constexpr double ROS23_C32 = 0x1.da827999fcef3p+2;
constexpr double ROS23_D = 0x1.2bec333018867p-2;

// PIController (OrdinaryDiffEqCore controllers.jl) with FastPower.fastpower:
//   q11 = fastpower(EEst, β1); q = clamp(q11 / fastpower(qold, β2) / γ, 1/qmax, 1/qmin)
//   accept: dtnew = dt / q, qold = max(EEst, qoldinit); reject: dt /= min(1/qmin, q11/γ)
// Evaluated for the latency of one lane's serial chain, bit-identical to the oracle:
//  * fastpower(EEst, β1) and the next fastpower(qold, β2) share fastlog2(Float32(EEst))
//    (qold = EEst whenever EEst > qoldinit) and their exp2s run side by side;
//  * q11 / fastpower(qold, β2) divides by a reciprocal refined when qold was set
//    (div_rcp: the IEEE quotient for these operand ranges, q11 ∈ [2^-21, 2^18]);
//  * the accept and reject step sizes are both formed, then selected.
struct PIControl {
    double qold_b2; // fastpower(qold, β2)
    double r_b2;    // its refined reciprocal
    double qb2_min; // fastpower(qoldinit, β2)
    double q11 = 0.0;
    ConstDiv by_gamma{CTL_GAMMA};
    __device__ __forceinline__ PIControl()
        : qold_b2(sbr_fastpow(CTL_QOLDMIN, CTL_BETA2)), r_b2(rcp_refined(qold_b2)), qb2_min(qold_b2)
    {
    }
    // one controller pass: returns the next dt; `accept` = ok && EEst <= 1 (EEst not NaN).
    // ok = false turns the pass into a no-op on the controller state (a step that the
    // caller discards).  One division: the accept (dt/q) and reject (dt/min(1/qmin, q11/γ))
    // denominators are selected first.
    __device__ __forceinline__ double next_dt(double EEst, double dt, double dtmax, double dtmin, bool& accept,
                                              bool ok = true)
    {
        const float L = sbr_fastlog2f((float)EEst);
        const double p1 = (double)sbr_exp2f_jl((float)CTL_BETA1 * L); // fastpower(EEst, β1)
        const double p2 = (double)sbr_exp2f_jl((float)CTL_BETA2 * L); // fastpower(EEst, β2)
        const bool zero = EEst == 0.0;
        // p1, q11 = fastpower(·, β1) ∈ [2^-18, 2^18]: finite, so the +Inf select of by_gamma is dropped
        const double qq = by_gamma.finite(div_rcp(p1, qold_b2, r_b2));
        const double qc = vmax(CTL_INV_QMAX, vmin(CTL_INV_QMIN, qq));
        const double q = zero ? CTL_INV_QMAX : qc;
        q11 = zero ? q11 : p1;
        accept = ok & (EEst <= 1.0);
        const double qrej = vmin(CTL_INV_QMIN, by_gamma.finite(q11));
        // dt / den with den in [1/qmax, 1/qmin] and dt in [dtmin, dtmax]: the division
        // sequence without its identity scaling steps (div_rcp), the IEEE quotient
        const double den = accept ? q : qrej;
        const double quot = div_rcp(dt, den, rcp_refined(den));
        // qold = max(EEst, qoldinit) on accept
        const double nb2 = EEst > CTL_QOLDMIN ? p2 : qb2_min;
        const double nr = rcp_refined(nb2);
        qold_b2 = accept ? nb2 : qold_b2;
        r_b2 = accept ? nr : r_b2;
        const double dta = vmax(vmin(dtmax, quot), dtmin);
        return accept ? dta : quot;
    }
};

// Rosenbrock23's dense output (_ode_interpolant, @muladd):
// y0 + dt·(c1·k1 + c2·k2), c1 = Θ(1 − Θ)/(1 − 2d), c2 = Θ(Θ − 2d)/(1 − 2d)
__device__ __forceinline__ double ros23_dense(double th, double dt, double y0, double k1, double k2)
{
    const double omd = 1.0 - 2.0 * ROS23_D;
    const double c1 = (th * (1.0 - th)) / omd;
    const double c2 = (th * fma(-2.0, ROS23_D, th)) / omd;
    return fma(dt, fma(c1, k1, c2 * k2), y0);
}

// the stages of an accepted step, for dense output (stiff: k[0], k[1] = Rosenbrock23's k1, k2)
struct StepK {
    double k[7];
    bool stiff;
};

struct OdeOut {
    int32_t naccept = 0, nreject = 0; // per solve (maxiters is clamped to INT32_MAX by the C API)
    int32_t nswitch = 0;
    uint32_t status = 0;
};

// Optional Sink::finish(const OdeOut&): called by the lane at the moment its solve ends (inside
// the step loop, with o final), so that a lane can publish its results while the other lanes
// of its wave are still integrating (the learning kernel's per-column readiness).
template <class S, class = void>
struct has_finish : std::false_type {};
template <class S>
struct has_finish<S, decltype(std::declval<S&>().finish(std::declval<const OdeOut&>()), void())> : std::true_type {};
template <class S>
__device__ __forceinline__ void sink_finish(S& s, const OdeOut& o)
{
    if constexpr (has_finish<S>::value) s.finish(o);
}

// dx/dt = βx(1 − x) (learning.jl:45-48) with ForwardDiff's ∂f/∂x through (β·x)·(1 − x):
// β·(1 − x) + (−1)·(β·x); autonomous, ∂f/∂t = 0
struct LogisticSys {
    double beta;
    __device__ __forceinline__ double eval(double, double x) const { return (beta * x) * (1.0 - x); }
    __device__ __forceinline__ void prepare(double, double) const {}
    __device__ __forceinline__ double stage(int, double, double x) const { return (beta * x) * (1.0 - x); }
    __device__ __forceinline__ void jac(double, double x, double& J, double& dT) const
    {
        J = beta * (1.0 - x) + (-1.0) * (beta * x);
        dT = 0.0;
    }
    __device__ __forceinline__ void accepted(double) const {}
    // k1 (FSAL: k7 of the last Tsit5 step, or Rosenbrock23's f(t+dt, u)) is bit for bit
    // the f(t, x) that initialize! re-evaluates after a switch: the same expression on the
    // same x (autonomous), so the re-evaluation is skipped
    static constexpr bool kFsalExact = true;
    static constexpr bool kPinTableau = true;
};

// ode_determine_initdt for a scalar ODE (order 5: dt₁ = (0.01/max(d₁,d₂))^(1/6));
// returns dt, sets k1 = f(T0, x0)
template <class Sys>
__device__ __forceinline__ double initdt_scalar(Sys& f, double T0, double T1, double x0, double rtol, double atol,
                                                double& k1)
{
    const double dtmax = T1 - T0;
    const double dtmin = sbr_jl_eps(dmax(fabs(T0), fabs(T1)));
    const double sk = fma(fabs(x0), rtol, atol);
    const double d0 = fabs(x0 / sk);
    k1 = f.eval(T0, x0);
    const double d1 = fabs(k1 / sk);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : (d0 / d1) / 100.0;
    dt0 = dmin(dt0, dtmax);
    double dt;
    if (dt0 < 10.0 * DBL_EPS) {
        dt = dmax(1e-6, dtmin);
    } else {
        const double u1 = fma(dt0, k1, x0);
        const double f1 = f.eval(T0 + dt0, u1);
        if (k1 == f1) {
            dt = dmax(dtmin, 100.0 * dt0);
        } else {
            const double d2 = fabs((f1 - k1) / sk) / dt0;
            const double md = dmax(d1, d2);
            const double dt1 = (md <= 1e-15) ? dmax(1e-6, dt0 * 1e-3) : sbr_pow_pos(0.01 / md, 1.0 / SBR_INITDT_DEN);
            dt = dmax(dtmin, dmin(dmin(100.0 * dt0, dt1), dtmax));
        }
    }
    return dt;
}

// The Tsit5 tableau held in VGPRs for the scalar loop: as literals the compiler keeps
// re-materialising the 64-bit constants it cannot hold in SGPRs (two s_mov_b32 each,
// every step, issued by the lone wave in series with its VALU work).
struct Tsit5Regs {
    double a31, a32, a41, a42, a43, a51, a52, a53, a54, a61, a62, a63, a64, a65, a71, a72, a73, a74, a75, a76, bt1, bt2, bt3, bt4, bt5, bt6, bt7;
    __device__ __forceinline__ Tsit5Regs()
        : a31(A31), a32(A32), a41(A41), a42(A42), a43(A43), a51(A51), a52(A52), a53(A53), a54(A54), a61(A61), a62(A62), a63(A63), a64(A64), a65(A65), a71(A71), a72(A72), a73(A73), a74(A74), a75(A75), a76(A76), bt1(BT1), bt2(BT2), bt3(BT3), bt4(BT4), bt5(BT5), bt6(BT6), bt7(BT7)
    {
        asm volatile("" : "+v"(a31));
        asm volatile("" : "+v"(a32));
        asm volatile("" : "+v"(a41));
        asm volatile("" : "+v"(a42));
        asm volatile("" : "+v"(a43));
        asm volatile("" : "+v"(a51));
        asm volatile("" : "+v"(a52));
        asm volatile("" : "+v"(a53));
        asm volatile("" : "+v"(a54));
        asm volatile("" : "+v"(a61));
        asm volatile("" : "+v"(a62));
        asm volatile("" : "+v"(a63));
        asm volatile("" : "+v"(a64));
        asm volatile("" : "+v"(a65));
        asm volatile("" : "+v"(a71));
        asm volatile("" : "+v"(a72));
        asm volatile("" : "+v"(a73));
        asm volatile("" : "+v"(a74));
        asm volatile("" : "+v"(a75));
        asm volatile("" : "+v"(a76));
        asm volatile("" : "+v"(bt1));
        asm volatile("" : "+v"(bt2));
        asm volatile("" : "+v"(bt3));
        asm volatile("" : "+v"(bt4));
        asm volatile("" : "+v"(bt5));
        asm volatile("" : "+v"(bt6));
        asm volatile("" : "+v"(bt7));
    }
};

// Literal tableau (no VGPRs held): for right-hand sides that need the registers more
// (lookup-heavy social / value-function RHS, which run near the 256-VGPR ceiling).
struct Tsit5Lits {
    static constexpr double a31 = A31;
    static constexpr double a32 = A32;
    static constexpr double a41 = A41;
    static constexpr double a42 = A42;
    static constexpr double a43 = A43;
    static constexpr double a51 = A51;
    static constexpr double a52 = A52;
    static constexpr double a53 = A53;
    static constexpr double a54 = A54;
    static constexpr double a61 = A61;
    static constexpr double a62 = A62;
    static constexpr double a63 = A63;
    static constexpr double a64 = A64;
    static constexpr double a65 = A65;
    static constexpr double a71 = A71;
    static constexpr double a72 = A72;
    static constexpr double a73 = A73;
    static constexpr double a74 = A74;
    static constexpr double a75 = A75;
    static constexpr double a76 = A76;
    static constexpr double bt1 = BT1;
    static constexpr double bt2 = BT2;
    static constexpr double bt3 = BT3;
    static constexpr double bt4 = BT4;
    static constexpr double bt5 = BT5;
    static constexpr double bt6 = BT6;
    static constexpr double bt7 = BT7;
};
// The stage coefficients a_ij in VGPRs and the error weights as literals (a right-hand side
// with room for 40 more VGPRs but not 54)
struct Tsit5RegsA {
    double a31, a32, a41, a42, a43, a51, a52, a53, a54, a61, a62, a63, a64, a65, a71, a72, a73, a74, a75, a76;
    static constexpr double bt1 = BT1;
    static constexpr double bt2 = BT2;
    static constexpr double bt3 = BT3;
    static constexpr double bt4 = BT4;
    static constexpr double bt5 = BT5;
    static constexpr double bt6 = BT6;
    static constexpr double bt7 = BT7;
    __device__ __forceinline__ Tsit5RegsA()
        : a31(A31), a32(A32), a41(A41), a42(A42), a43(A43), a51(A51), a52(A52), a53(A53), a54(A54), a61(A61), a62(A62), a63(A63), a64(A64), a65(A65), a71(A71), a72(A72), a73(A73), a74(A74), a75(A75), a76(A76)
    {
        asm volatile("" : "+v"(a31));
        asm volatile("" : "+v"(a32));
        asm volatile("" : "+v"(a41));
        asm volatile("" : "+v"(a42));
        asm volatile("" : "+v"(a43));
        asm volatile("" : "+v"(a51));
        asm volatile("" : "+v"(a52));
        asm volatile("" : "+v"(a53));
        asm volatile("" : "+v"(a54));
        asm volatile("" : "+v"(a61));
        asm volatile("" : "+v"(a62));
        asm volatile("" : "+v"(a63));
        asm volatile("" : "+v"(a64));
        asm volatile("" : "+v"(a65));
        asm volatile("" : "+v"(a71));
        asm volatile("" : "+v"(a72));
        asm volatile("" : "+v"(a73));
        asm volatile("" : "+v"(a74));
        asm volatile("" : "+v"(a75));
        asm volatile("" : "+v"(a76));
    }
};
// PIN: 0 = literals, 1 = the whole tableau in VGPRs, 2 = the stage coefficients only
template <int PIN>
struct Tsit5Tab : Tsit5Regs {};
template <>
struct Tsit5Tab<0> : Tsit5Lits {};
template <>
struct Tsit5Tab<2> : Tsit5RegsA {};

// Scalar AutoTsit5(Rosenbrock23()) on (0, T1) from x0.  Sys provides
//   double eval(double t, double x)                       f at any (t, x)
//   void   prepare(double t, double dt)                   before the Tsit5 stages of a step
//   double stage(int s, double ts, double x)              Tsit5 stage s = 1..6 (k2..k7) at time ts
//   void   jac(double t, double x, double& J, double& dT) ForwardDiff ∂f/∂x, ∂f/∂t
//   void   accepted(double t)                             after an accepted step
//   static constexpr bool kFsalExact                      f(t, x) == the carried k1 bit for bit
//   static constexpr bool/int kPinTableau                 the Tsit5 tableau in VGPRs: 0 / false literals,
//                                                          1 / true all (Tsit5Regs), 2 the a_ij (Tsit5RegsA)
// Sink provides
//   bool start(double t0, double x0)                      the first knot; false = stop
//   bool step(bool acc, double tprev, double tn, double dt, double y0, double y1, const StepK& k, bool exact)
//        called after EVERY attempted step (acc: accepted — the sink must ignore rejected
//        ones); exact: tn == tprev + dt (no snap to T1); false = stop.
// The 64 lanes of a wave integrate 64 different ODEs whose steps are accepted and
// rejected independently, so the step bookkeeping is branch-free (state updates by
// select, knots written unconditionally at the fill index): a divergent accept / reject
// branch would run both sides and serialise exec-mask updates on the lane's chain.
template <class S, class = void>
struct accept_first : std::false_type {};
template <class S>
struct accept_first<S, std::void_t<decltype(S::kAcceptFirst)>> : std::bool_constant<S::kAcceptFirst> {};

template <class Sys, class Sink>
__device__ __forceinline__ void ode_scalar(Sys& f, Sink& sink, double T1, double x0, double rtol, double atol,
                                           int64_t maxiters, OdeOut& o)
{
    const double T0 = 0.0;
    const double dtmax = T1 - T0;
    const double dtmin = sbr_jl_eps(dmax(fabs(T0), fabs(T1)));
    double k1;
    double dt = initdt_scalar(f, T0, T1, x0, rtol, atol, k1);
    const double snap = 100.0 * sbr_jl_eps(T1);
    double t = T0, x = x0;
    double eig = 1.0; // integrator.eigen_est = 1/oneunit(t) at init
    PIControl pc;
    AutoSwitch as;
    const Tsit5Tab<(int)Sys::kPinTableau> cf;
    if (!sink.start(t, x)) { sink_finish(sink, o); return; }
    if (!(t < T1)) { sink_finish(sink, o); return; }
    if (maxiters < 1) { o.status |= SBR_ODE_MAXITERS; sink_finish(sink, o); return; }
    // One loop exit, tested at the bottom: the reference's early exits (DtLessThanMin before
    // the step, a NaN trial state after it) compute the step and discard it (ok = false: no
    // knot, no controller / state update, not counted), and the maxiters test of the next
    // loopheader is made at the end of this iteration.  A divergent multi-exit loop costs
    // every lane the exit-mask bookkeeping of all exits on every step.
    int64_t iter = 0;
    uint32_t why = 0; // status bits of the exit (an int, not loop-carried bools)
    for (;;) {
        ++iter;
        // initialize! of the new algorithm: fsalfirst = f(uprev, t)
        if (Sys::kFsalExact) {
            (void)as.choose(eig, dt);
        } else if (as.choose(eig, dt)) {
            k1 = f.eval(t, x);
        }
        dt = vmin(dtmax, dt);
        dt = vmax(dt, dtmin);
        dt = vmin(dt, T1 - t);
        const bool dtfail = (dt <= dtmin) & (t + dt < T1); // DtLessThanMin
        StepK K;
        double u, fnew, EEst;
        if (as.stiff) {
            // ---- Rosenbrock23 (perform_step!, @muladd), 1×1 W: the solves are divisions ----
            K.stiff = true;
            double J, dT;
            f.jac(t, x, J, dT);
            const double dtg = dt * ROS23_D;
            const double invdtg = 1.0 / dtg, neginvdtg = -(1.0 / dtg);
            const double dto2 = dt / 2.0, dto6 = dt / 6.0;
            const double W = fma(-1.0, invdtg, J);
            const double r1 = k1 + dtg * dT;
            const double s1 = (r1 / W) * neginvdtg;
            const double tmp = fma(dto2, s1, x);
            const double f1 = f.eval(t + dto2, tmp);
            const double s2 = fma((f1 - s1) / W, neginvdtg, s1);
            u = fma(dt, s2, x);
            fnew = f.eval(t + dt, u);
            const double r3 = fma(dt, dT, fma(-2.0, s1 - k1, fma(-ROS23_C32, s2 - f1, fnew)));
            const double s3 = (r3 / W) * neginvdtg;
            const double ut = dto6 * (fma(-2.0, s2, s1) + s3);
            EEst = fabs(ut / fma(dmax(fabs(x), fabs(u)), rtol, atol));
            K.k[0] = s1;
            K.k[1] = s2;
            eig = fabs(J);
        } else {
            // ---- Tsit5 (perform_step!, Tsit5ConstantCache, @muladd) ----
            K.stiff = false;
            f.prepare(t, dt);
            double tmp = fma(dt * A21, k1, x);
            const double k2 = f.stage(1, fma(C1, dt, t), tmp);
            tmp = fma(dt, fma(cf.a31, k1, cf.a32 * k2), x);
            const double k3 = f.stage(2, fma(C2, dt, t), tmp);
            tmp = fma(dt, fma(cf.a41, k1, fma(cf.a42, k2, cf.a43 * k3)), x);
            const double k4 = f.stage(3, fma(C3, dt, t), tmp);
            tmp = fma(dt, fma(cf.a51, k1, fma(cf.a52, k2, fma(cf.a53, k3, cf.a54 * k4))), x);
            const double k5 = f.stage(4, fma(C4, dt, t), tmp);
            const double tmp6 = fma(dt, fma(cf.a61, k1, fma(cf.a62, k2, fma(cf.a63, k3, fma(cf.a64, k4, cf.a65 * k5)))), x);
            const double k6 = f.stage(5, t + dt, tmp6);
            u = fma(dt, fma(cf.a71, k1, fma(cf.a72, k2, fma(cf.a73, k3, fma(cf.a74, k4, fma(cf.a75, k5, cf.a76 * k6))))), x);
            const double k7 = f.stage(6, t + dt, u);
            const double eigr = fabs((k7 - k6) / (u - tmp6));
            const double ut =
                dt * fma(cf.bt1, k1, fma(cf.bt2, k2, fma(cf.bt3, k3, fma(cf.bt4, k4, fma(cf.bt5, k5, fma(cf.bt6, k6, cf.bt7 * k7))))));
            EEst = fabs(ut / fma(dmax(fabs(x), fabs(u)), rtol, atol));
            fnew = k7;
            K.k[0] = k1; K.k[1] = k2; K.k[2] = k3; K.k[3] = k4; K.k[4] = k5; K.k[5] = k6; K.k[6] = k7;
            eig = (eigr != eigr) ? (double)NAN : eigr;
        }
        const bool nan = EEst != EEst; // NaN trial state (ReturnCode.Unstable)
        const bool ok = (!dtfail) & (!nan);
        bool acc;
        const double dtn = pc.next_dt(EEst, dt, dtmax, dtmin, acc, ok);
        const double tdt = t + dt;
        const double tn = fabs(tdt - T1) < snap ? T1 : tdt; // fixed_t_for_floatingpoint_error!
        // a Sys whose accepted() issues loads (SocialRhsRing's ring refill) takes it before the
        // knot's stores, so that the refill's wait does not drain them (the lookups are exact
        // whatever the window's position: the same knot values either way)
        if constexpr (accept_first<Sys>::value) { if (acc) f.accepted(tn); }
        const bool go = sink.step(acc, t, tn, dt, x, u, K, tn == tdt);
        if constexpr (!accept_first<Sys>::value) { if (acc) f.accepted(tn); }
        t = acc ? tn : t;
        x = acc ? u : x;
        k1 = acc ? fnew : k1;
        dt = ok ? dtn : dt;
        o.naccept += acc ? 1 : 0;
        o.nreject += (ok & !acc) ? 1 : 0;
        // bitwise (not short-circuit) logic: no branches for the compiler to form; the
        // exit reason is turned into status bits once, after the loop
        const bool badt = ok & go & !((dt > 0.0) & (fabs(dt) < (double)INFINITY));
        const bool more = t < T1;
        const bool maxit = ok & go & !badt & more & (iter >= maxiters);
        const bool fail = (!ok) | badt;
        why = (fail ? SBR_ODE_FAILED : 0u) | (maxit ? SBR_ODE_MAXITERS : 0u);
        if (fail | (!go) | (!more) | maxit) {
            if constexpr (has_finish<Sink>::value) {
                o.status |= why;
                o.nswitch = as.nswitch;
                if (as.nswitch > 0) o.status |= SBR_STIFF_SWITCH;
                sink.finish(o);
            }
            break;
        }
    }
    o.status |= why;
    o.nswitch = as.nswitch;
    if (as.nswitch > 0) o.status |= SBR_STIFF_SWITCH;
}

}  // namespace sbr
