// sbr_hetero.hip — gfx950 kernels for the heterogeneity extension (K coupled
// learning groups), src/extensions/heterogeneity/.
//
//   learn_hetero_wave_kernel<K>   one wave per parameter column (lane k = group k):
//                                 FP64 AutoTsit5(Rosenbrock23()) on
//                                 dG_k/dt = (1−G_k) β_k Σ_j dist_j G_j with the
//                                 RMS error norm over K components
//                                 (heterogeneity_learning.jl:49-94), pdfs
//                                 (compute_pdf_hetero :114-134) and the K hazard
//                                 rates on the explicit-grid τ̄ (solver.jl:163-164:
//                                 η always appended) streamed per knot.
//   equilibrium_hetero_kernel<K>  one lane per (column, u): K crossing scans,
//                                 the dist-weighted ξ bisection on [0, 2 max τ̄_OUT]
//                                 (compute_ξ_hetero :48-144), the multimodality
//                                 validity check (:175-210) and AW_max over the
//                                 whole learning grid (get_AW_hetero :316-375).
// Knot times are staged in LDS; G (AoS [knot][K]) and HR ([K][τ̄]) stay in HBM/L2.
// Bit-exact against oracle/sbr_oracle.c (sbro_sweep_hetero).
#include "sbr_device.h"
#include "sbr_kernels.h"
#include "sbr_ode.h"
#include "sbr_scan.h"

namespace sbr {

template <int K>
__device__ __forceinline__ double omega(const double* __restrict__ dist, const double* I)
{
    double w = dist[0] * I[0];
#pragma unroll
    for (int j = 1; j < K; j++) w = w + dist[j] * I[j];
    return w;
}

template <int K>
__device__ __forceinline__ void rhs(const double* __restrict__ dist, const double* b, const double* I, double* du)
{
    const double w = omega<K>(dist, I);
#pragma unroll
    for (int k = 0; k < K; k++) du[k] = ((1.0 - I[k]) * b[k]) * w;
}

template <int K>
__device__ __forceinline__ double rms(const double* v)
{
    if (K == 1) return fabs(v[0]);
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < K; i++) s = s + v[i] * v[i];
    return sqrt(s / (double)K);
}

// ForwardDiff jacobian of rhs (oracle jac_hetero): b_k = (1 − I_k)·β_k,
// J_kj = dist_j·b_k (j ≠ k), J_kk = (−β_k)·ω + dist_k·b_k; autonomous (∂f/∂t = 0)
template <int K>
__device__ __forceinline__ void jac(const double* __restrict__ dist, const double* b, const double* I, double* J)
{
    const double w = omega<K>(dist, I);
#pragma unroll
    for (int k = 0; k < K; k++) {
        const double bk = (1.0 - I[k]) * b[k];
#pragma unroll
        for (int j = 0; j < K; j++) J[k * K + j] = (j == k) ? (-b[k]) * w + dist[k] * bk : dist[j] * bk;
    }
}

// opnorm(J, Inf) (NaN-propagating max of the row sums): Rosenbrock23's eigen_est
template <int K>
__device__ __forceinline__ double opnorm_inf(const double* J)
{
    double nrm = 0.0;
#pragma unroll
    for (int i = 0; i < K; i++) {
        double s = 0.0;
#pragma unroll
        for (int j = 0; j < K; j++) s = s + fabs(J[i * K + j]);
        nrm = (nrm != nrm || s != s) ? (double)NAN : (s > nrm ? s : nrm);
    }
    return nrm;
}

// ---------------------------------------------------------------------------
// learn_hetero_wave_kernel<K>: one wave per column, lane k = group k
// ---------------------------------------------------------------------------
// The oracle's AutoTsit5(Rosenbrock23()) solve (sbro_learn_hetero), bit for bit, laid out for the
// lone wave's serial chain (one lane per column, 64 columns per wave, ran both the Tsit5 and the
// Rosenbrock23 branch whenever the columns disagreed: 85 -> 28–32 ms per config-4 grid):
//  * lane k holds component k of every stage vector and row k of W; the couplings (ω, the
//    RMS error norm, the eigen estimates, the LU's pivot column and pivot row, the
//    substitutions) read the other lanes' values with v_readlane into SGPRs and fold them
//    in the oracle's order, so every sum and max is the same left fold;
//  * the step control (t, dt, controller, AutoSwitch, knot counters) is wave-uniform: no
//    divergence between the columns' Tsit5 and Rosenbrock23 phases (with 64 columns per
//    wave both branches ran whenever the columns disagreed);
//  * a row interchange is a uniform branch taken only when the pivot leaves the diagonal.
// Lanes >= K shadow component K-1's arithmetic and never store or get read.
// (Four columns per wave, one 16-lane row each with DPP row broadcasts, was bit-identical and
// slower: a wave runs until its slowest column and executes both branches while its rows
// disagree, 42.4 -> 45.2 ms per config-4 step, profiles/experiments/r04_s_*.)
__device__ __forceinline__ double wave_bcast(double v, int l)
{
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
    return __hiloint2double(hi, lo);
}

template <int K>
struct WaveRow {
    const int lane; // row / component index of this lane (lanes >= K: K - 1's shadow)
    const int kk;
    const double bk, dk; // β_k, dist_k
    const double* __restrict__ dist;
    __device__ __forceinline__ WaveRow(int l, const double* __restrict__ betas_c, const double* __restrict__ d)
        : lane(l), kk(l < K ? l : K - 1), bk(betas_c[kk]), dk(d[kk]), dist(d)
    {
    }
    // ω = dist_0·I_0 + dist_1·I_1 + … (rhs_hetero's left fold; each product formed in its lane)
    __device__ __forceinline__ double omega(double I) const
    {
        const double pr = dk * I;
        double w = wave_bcast(pr, 0);
#pragma unroll
        for (int j = 1; j < K; j++) w = w + wave_bcast(pr, j);
        return w;
    }
    __device__ __forceinline__ double rhs(double I) const { return ((1.0 - I) * bk) * omega(I); }
    // sqrt(Σ v_k² / K), the sum from 0.0 in component order
    __device__ __forceinline__ double rms(double v) const
    {
        if (K == 1) return wave_bcast(fabs(v), 0);
        const double sq = v * v;
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < K; i++) s = s + wave_bcast(sq, i);
        return sqrt(s / (double)K);
    }
};

// Row-distributed K×K LU (generic_lufact! / getrs, the oracle's lu_factor / lu_solve operation
// sequence): lane i holds row i of A.
template <int K>
struct WaveLU {
    double A[K];
    int piv[K]; // wave-uniform
    __device__ __forceinline__ void factor(int lane)
    {
#pragma unroll
        for (int k = 0; k < K; k++) {
            double pv = wave_bcast(A[k], k);
            double amax = fabs(pv);
            int kp = k;
#pragma unroll
            for (int i = k + 1; i < K; i++) {
                const double ai = wave_bcast(A[k], i);
                if (fabs(ai) > amax) { kp = i; amax = fabs(ai); pv = ai; }
            }
            piv[k] = kp;
            if (pv != 0.0) {
                if (kp != k) {
#pragma unroll
                    for (int j = 0; j < K; j++) {
                        const double vk = wave_bcast(A[j], k), vp = wave_bcast(A[j], kp);
                        A[j] = lane == k ? vp : (lane == kp ? vk : A[j]);
                    }
                }
                const double inv = 1.0 / pv; // A[k][k] after the interchange
                const double sc = A[k] * inv;
                A[k] = lane > k ? sc : A[k];
            }
#pragma unroll
            for (int j = k + 1; j < K; j++) {
                const double akj = wave_bcast(A[j], k);
                const double v = A[j] - A[k] * akj;
                A[j] = lane > k ? v : A[j];
            }
        }
    }
    // b: this lane's component of the right-hand side, overwritten with the solution's
    __device__ __forceinline__ void solve(double& b, int lane) const
    {
#pragma unroll
        for (int k = 0; k < K; k++) {
            const int kp = piv[k];
            if (kp != k) {
                const double x = wave_bcast(b, k), y = wave_bcast(b, kp);
                b = lane == k ? y : (lane == kp ? x : b);
            }
        }
#pragma unroll
        for (int j = 0; j < K; j++) {
            const double a = -wave_bcast(b, j);
            const double v = fma(a, A[j], b);
            b = lane > j ? v : b;
        }
#pragma unroll
        for (int j = K - 1; j >= 0; j--) {
            const double bj = wave_bcast(b / A[j], j); // lane j: b_j / A[j][j]
            b = lane == j ? bj : b;
            const double v = fma(-bj, A[j], b);
            b = lane < j ? v : b;
        }
    }
};

// waves (columns) per learning workgroup.  Config-4 step, same-call A/Bs (r05_kk, r05_ll): one
// wave per workgroup 43.4 ms (45.7–46.0 with this kernel's wave indexing), 4 waves (one per SIMD
// of a CU) 42.2–42.3, 2 waves 51.6 (r05_nn), 8 waves (two per SIMD: the learning becomes the critical path) 47.6
constexpr int kHetLearnWG = 4;
template <int K>
__global__ __launch_bounds__(64 * kHetLearnWG) void learn_hetero_wave_kernel(const double* __restrict__ betas,
                                                               const double* __restrict__ dist,
                                                               const double* __restrict__ eta,
                                                               const double* __restrict__ t_end, LearnArgs a,
                                                               HeteroBufs L)
{
    const int c = blockIdx.x * kHetLearnWG + (int)(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (c >= a.n_beta) return; // a whole wave (the column index is wave-uniform)
    const bool act = lane < K;
    const WaveRow<K> R(lane, betas + (size_t)c * K, dist);
    const double ETA = eta[c], T1 = t_end[c], T0 = 0.0;
    const size_t cap = (size_t)L.cap;
    double* __restrict__ T = L.t + (size_t)c * cap;
    double* __restrict__ Gv = L.G + (size_t)c * cap * K;
    double* __restrict__ H = L.hr + ((size_t)c * K + R.kk) * cap;
    double* __restrict__ HI = L.hrI + ((size_t)c * K + R.kk) * cap;
    uint32_t st = 0;
    bool argok = ETA > 0.0 && T1 > T0;
#pragma unroll
    for (int k = 0; k < K; k++) argok = argok && (wave_bcast(R.bk, k) > 0.0);
    if (!argok) {
        if (lane == 0) {
            L.status[c] = SBR_ARG_INVALID;
            L.n_knots[c] = 0; L.n_tau[c] = 0; L.n_le[c] = 0; L.n_accept[c] = 0; L.n_reject[c] = 0;
        }
        return;
    }
    const double x0 = a.x0, rtol = a.rtol, atol = a.atol, p = a.p, lam = a.lam;
    const double dtmax = T1 - T0;
    const double dtmin = sbr_jl_eps(dmax(fabs(T0), fabs(T1)));
    double x, k1, k2, k3, k4, k5, k6, k7, tmp, tmp6, u;

    // ---- ode_determine_initdt ----
    x = x0;
    const double sk = fma(fabs(x0), rtol, atol);
    const double d0 = R.rms(x0 / sk);
    k1 = R.rhs(x);
    const double d1 = R.rms(k1 / sk);
    double dt0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : (d0 / d1) / 100.0;
    dt0 = dmin(dt0, dtmax);
    double dt;
    if (dt0 < 10.0 * DBL_EPS) {
        dt = dmax(1e-6, dtmin);
    } else {
        u = fma(dt0, k1, x0);
        k7 = R.rhs(u);
        bool same = true;
#pragma unroll
        for (int k = 0; k < K; k++) same = same && (__builtin_amdgcn_readlane((int)(k1 == k7), k) != 0);
        if (same) {
            dt = dmax(dtmin, 100.0 * dt0);
        } else {
            const double d2 = R.rms((k7 - k1) / sk) / dt0;
            const double md = dmax(d1, d2);
            const double dt1 = (md <= 1e-15) ? dmax(1e-6, dt0 * 1e-3) : sbr_pow_pos(0.01 / md, 1.0 / SBR_INITDT_DEN);
            dt = dmax(dtmin, dmin(dmin(100.0 * dt0, dt1), dtmax));
        }
    }

    // ---- knot sink: (t, G_k) + this lane's streamed hazard terms; g = f(t, x)_k is the
    // FSAL value of the step that produced the knot (the same expression on the same x) ----
    int n = 0, m = 0;
    double tprev = 0.0, Ik = 0.0, eprev = 0.0, gprev = 0.0;
    bool past = false, done = false;
    auto push = [&](double t, double xs, double g) {
        if (n >= L.lim) { st |= SBR_KNOT_OVERFLOW; done = true; return; }
        if (lane == 0) T[n] = t;
        if (act) Gv[(size_t)n * K + lane] = xs;
        if (!past) {
            if (t <= ETA) {
                const double E = sbr_exp(lam * t);
                const double e = E * g;
                Ik = (m == 0) ? 0.0 : Ik + (0.5 * (eprev + e)) * (t - tprev);
                if (act) { H[m] = (p * E) * g; HI[m] = Ik; }
                eprev = e;
                gprev = g;
                m++;
                tprev = t;
            } else {
                past = true; // η always appended (explicit grid): pdf(η) on bracket [n-1, n]
                const double d = (ETA - tprev) / (t - tprev);
                const double E = sbr_exp(lam * ETA);
                const double pe = gprev * (1.0 - d) + g * d;
                const double e = E * pe;
                Ik = Ik + (0.5 * (eprev + e)) * (ETA - tprev);
                if (act) { H[m] = (p * E) * pe; HI[m] = Ik; }
                m++;
            }
        }
        n++;
    };

    const double snap = 100.0 * sbr_jl_eps(T1);
    double t = T0;
    double eig = 1.0; // integrator.eigen_est at init
    PIControl pc;
    AutoSwitch as;
    const Tsit5Tab<0> cf; // literals (the tableau in VGPRs: 103 -> 157 VGPRs, step 42.7 -> 46.6 ms, r05_x)
    int naccept = 0, nreject = 0;
    push(t, x, k1);
    int64_t iter = 0;
    while (t < T1 && !done) {
        if (++iter > a.maxiters) { st |= SBR_ODE_MAXITERS; break; }
        (void)as.choose(eig, dt); // initialize!: fsalfirst = f(uprev, t) == k1 bit for bit (autonomous)
        dt = dmin(dtmax, dt);
        dt = dmax(dt, dtmin);
        dt = dmin(dt, T1 - t);
        if (dt <= dtmin && t + dt < T1) { st |= SBR_ODE_FAILED; break; } // DtLessThanMin
        double EEst;
        if (as.stiff) {
            // ---- Rosenbrock23 (perform_step!, Rosenbrock23Cache, @muladd); k7 <- fsallast ----
            const double dtg = dt * ROS23_D;
            const double invdtg = 1.0 / dtg, neginvdtg = -(1.0 / dtg);
            const double dto2 = dt / 2.0, dto6 = dt / 6.0;
            WaveLU<K> W;
            {
                // ForwardDiff jacobian row k: J_kj = dist_j·b_k, J_kk = (−β_k)·ω + dist_k·b_k
                const double w = R.omega(x);
                const double bkx = (1.0 - x) * R.bk;
                const double dg = (-R.bk) * w + R.dk * bkx;
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < K; j++) {
                    W.A[j] = (j == lane) ? dg : dist[j] * bkx;
                    s = s + fabs(W.A[j]);
                }
                // opnorm(J, Inf): NaN-propagating max of the row sums, in row order
                double nrm = 0.0;
#pragma unroll
                for (int i = 0; i < K; i++) {
                    const double si = wave_bcast(s, i);
                    nrm = (nrm != nrm || si != si) ? (double)NAN : (si > nrm ? si : nrm);
                }
                eig = nrm;
#pragma unroll
                for (int j = 0; j < K; j++) W.A[j] = (j == lane) ? fma(-1.0, invdtg, W.A[j]) : W.A[j];
            }
            W.factor(lane);
            double r = k1 + dtg * 0.0; // fsalfirst + dt·d·∂f/∂t
            W.solve(r, lane);
            const double s1 = r * neginvdtg;
            tmp = fma(dto2, s1, x);
            const double f1 = R.rhs(tmp);
            r = f1 - s1;
            W.solve(r, lane);
            const double s2 = fma(r, neginvdtg, s1);
            u = fma(dt, s2, x);
            k7 = R.rhs(u);
            r = fma(dt, 0.0, fma(-2.0, s1 - k1, fma(-ROS23_C32, s2 - f1, k7)));
            W.solve(r, lane);
            const double s3 = r * neginvdtg;
            const double ut = dto6 * (fma(-2.0, s2, s1) + s3);
            EEst = R.rms(ut / fma(dmax(fabs(x), fabs(u)), rtol, atol));
        } else {
            const double a21 = dt * A21;
            tmp = fma(a21, k1, x);
            k2 = R.rhs(tmp);
            tmp = fma(dt, fma(cf.a31, k1, cf.a32 * k2), x);
            k3 = R.rhs(tmp);
            tmp = fma(dt, fma(cf.a41, k1, fma(cf.a42, k2, cf.a43 * k3)), x);
            k4 = R.rhs(tmp);
            tmp = fma(dt, fma(cf.a51, k1, fma(cf.a52, k2, fma(cf.a53, k3, cf.a54 * k4))), x);
            k5 = R.rhs(tmp);
            tmp6 = fma(dt, fma(cf.a61, k1, fma(cf.a62, k2, fma(cf.a63, k3, fma(cf.a64, k4, cf.a65 * k5)))), x);
            k6 = R.rhs(tmp6);
            u = fma(dt, fma(cf.a71, k1, fma(cf.a72, k2, fma(cf.a73, k3, fma(cf.a74, k4, fma(cf.a75, k5, cf.a76 * k6))))), x);
            k7 = R.rhs(u);
            const double rr = fabs((k7 - k6) / (u - tmp6));
            double e = 0.0;
            bool e_nan = false;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const double v = wave_bcast(rr, k);
                if (v != v) e_nan = true;
                else if (v > e) e = v;
            }
            eig = e_nan ? (double)NAN : e;
            const double ut = dt * fma(cf.bt1, k1, fma(cf.bt2, k2, fma(cf.bt3, k3, fma(cf.bt4, k4,
                                       fma(cf.bt5, k5, fma(cf.bt6, k6, cf.bt7 * k7))))));
            EEst = R.rms(ut / fma(dmax(fabs(x), fabs(u)), rtol, atol));
        }
        if (EEst != EEst) { st |= SBR_ODE_FAILED; break; } // NaN trial state (ReturnCode.Unstable)
        bool acc;
        const double dtn = pc.next_dt(EEst, dt, dtmax, dtmin, acc);
        if (acc) {
            naccept++;
            double tn = t + dt;
            if (fabs(tn - T1) < snap) tn = T1;
            t = tn;
            x = u;
            k1 = k7;
            dt = dtn;
            push(t, x, k1);
        } else {
            nreject++;
            dt = dtn;
        }
        if (!(dt > 0.0) || !isfinite(dt)) { st |= SBR_ODE_FAILED; break; }
    }
    if (as.nswitch > 0) st |= SBR_STIFF_SWITCH;
    int n_le = m;
    if (past) {
        n_le = m - 1;
    } else if (!(st & SBR_KNOT_OVERFLOW)) {
        // no knot beyond η: pdf(η) exists only if the last knot is η itself
        if (n >= 2 && tprev == ETA) {
            const double E = sbr_exp(lam * ETA);
            // bracket clamps to [n-2, n-1] with δ = 1: gprev*(1-1) ... = g_{n-1}
            const double pe = 0.0 + gprev * 1.0;
            if (act) { H[m] = (p * E) * pe; HI[m] = Ik; }
            m++;
        } else {
            st |= SBR_OOB;
        }
    }
    if (m > 0 && !(st & SBR_OOB)) {
        // normalisation hr = p·e^{λτ̄}g / (p·I(τ̄) + (1 − p)·I(η)), all 64 lanes over each group's row
        __threadfence_block();
        const double omp = 1.0 - p;
        double* __restrict__ Hc = L.hr + (size_t)c * K * cap;
        const double* __restrict__ HIc = L.hrI + (size_t)c * K * cap;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double Ieta = HIc[(size_t)k * cap + m - 1];
            for (int i = lane; i < m; i += 64)
                Hc[(size_t)k * cap + i] = Hc[(size_t)k * cap + i] / ((p * HIc[(size_t)k * cap + i]) + (omp * Ieta));
        }
    }
    if (lane == 0) {
        L.n_knots[c] = n;
        L.n_tau[c] = m;
        L.n_le[c] = n_le;
        L.status[c] = st;
        L.n_accept[c] = naccept;
        L.n_reject[c] = nreject;
    }
}

// The K hazards (heterogeneity_solver.jl:255: hazard_rate on the explicit grid = the learning
// knots, η always appended) of a column whose knots and group CDFs are already in L — a
// LearningResultsHetero the caller holds (sbr_hetero_equilibrium_on_knots).  The streamed hazard
// of learn_hetero_wave_kernel, operation for operation, over that grid: pdf_k at a knot is
// compute_pdf_hetero (heterogeneity_learning.jl:114-134), rhs_k of the knot's state — the FSAL
// value the learning kernel streams.  One wave per column, lane k = group k.  Knots starting
// after η make pdf(η) the interpolant's BoundsError (SBR_OOB) like an η past the last knot.
template <int K>
__global__ __launch_bounds__(64) void hazard_hetero_kernel(const double* __restrict__ betas,
                                                           const double* __restrict__ dist,
                                                           const double* __restrict__ eta, LearnArgs a, HeteroBufs L)
{
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const bool act = lane < K;
    const WaveRow<K> R(lane, betas + (size_t)c * K, dist);
    const double ETA = eta[c];
    const size_t cap = (size_t)L.cap;
    const double* __restrict__ T = L.t + (size_t)c * cap;
    const double* __restrict__ Gv = L.G + (size_t)c * cap * K;
    double* __restrict__ H = L.hr + ((size_t)c * K + R.kk) * cap;
    double* __restrict__ HI = L.hrI + ((size_t)c * K + R.kk) * cap;
    const int n = L.n_knots[c];
    uint32_t st = L.status[c];
    const double p = a.p, lam = a.lam;
    int m = 0;
    double tprev = 0.0, Ik = 0.0, eprev = 0.0, gprev = 0.0;
    bool past = false;
    for (int i = 0; i < n && !past; i++) {
        const double t = T[i];
        const double g = R.rhs(Gv[(size_t)i * K + R.kk]);
        if (t <= ETA) {
            const double E = sbr_exp(lam * t);
            const double e = E * g;
            Ik = (m == 0) ? 0.0 : Ik + (0.5 * (eprev + e)) * (t - tprev);
            if (act) { H[m] = (p * E) * g; HI[m] = Ik; }
            eprev = e;
            gprev = g;
            m++;
            tprev = t;
        } else if (m == 0) {
            st |= SBR_OOB; // η before the first knot
            break;
        } else {
            past = true; // pdf(η) on bracket [i-1, i]
            const double d = (ETA - tprev) / (t - tprev);
            const double E = sbr_exp(lam * ETA);
            const double pe = gprev * (1.0 - d) + g * d;
            const double e = E * pe;
            Ik = Ik + (0.5 * (eprev + e)) * (ETA - tprev);
            if (act) { H[m] = (p * E) * pe; HI[m] = Ik; }
            m++;
        }
    }
    int n_le = m;
    if (past) {
        n_le = m - 1;
    } else if (!(st & SBR_OOB)) {
        if (n >= 2 && tprev == ETA) { // η is the last knot: pdf(η) = its value
            const double E = sbr_exp(lam * ETA);
            const double pe = 0.0 + gprev * 1.0;
            if (act) { H[m] = (p * E) * pe; HI[m] = Ik; }
            m++;
        } else {
            st |= SBR_OOB;
        }
    }
    if (m > 0 && !(st & SBR_OOB)) {
        __threadfence_block();
        const double omp = 1.0 - p;
        double* __restrict__ Hc = L.hr + (size_t)c * K * cap;
        const double* __restrict__ HIc = L.hrI + (size_t)c * K * cap;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double Ieta = HIc[(size_t)k * cap + m - 1];
            for (int i = lane; i < m; i += 64)
                Hc[(size_t)k * cap + i] = Hc[(size_t)k * cap + i] / ((p * HIc[(size_t)k * cap + i]) + (omp * Ieta));
        }
    }
    if (lane == 0) {
        L.n_tau[c] = (st & SBR_OOB) ? 0 : m;
        L.n_le[c] = (st & SBR_OOB) ? 0 : n_le;
        L.status[c] = st;
    }
}

// ---------------------------------------------------------------------------
// per-point solve
// ---------------------------------------------------------------------------
template <int K, class PT>
struct HCol {
    PT T;                       // knot times (LDS or global)
    const double* __restrict__ G;   // [n][K]
    const double* __restrict__ H;   // [K][cap]
    int n, ntau, nle;
    size_t cap;
    double ETA, T1;
    const double* __restrict__ hsum; // [2][K][nblk] per-64 HR block max / min (LDS), or null
    int nblk;
    __device__ __forceinline__ double tau(int i) const { return i < nle ? T[i] : ETA; }
    __device__ __forceinline__ double g(int j, int k) const { return G[(size_t)j * K + k]; }
    // Interpolations gridded-linear value of group k on bracket j (clamped)
    __device__ __forceinline__ double lerp(int j, int k, double x) const
    {
        if (j > n - 2) j = n - 2;
        if (j < 0) j = 0;
        const double d = (x - T[j]) / (T[j + 1] - T[j]);
        return g(j, k) * (1.0 - d) + g(j + 1, k) * d;
    }
};

constexpr int kHetUbcBits = 16; // bound-code width (8: 29.8 ms alone, the 1/256 window recomputes)
typedef unsigned short ubc_t;
template <int K, class PT>
__device__ __forceinline__ void solve_hetero_point(const HCol<K, PT>& C, const double* __restrict__ dist,
                                                   const double u, const double kappa, const int max_iters,
                                                   const double tolerance, const uint32_t lbits, double& xi_o,
                                                   double& aw_o, double& tol_o, uint32_t& st_o, int& it_o,
                                                   double* tin, double* tout, const bool mono, const int diag,
                                                   double* __restrict__ aw_path, const double env, const bool sep,
                                                   const int koff,
                                                   double* __restrict__ tin_g, double* __restrict__ tout_g,
                                                   ubc_t* __restrict__ ubc = nullptr, const int ubc_stride = 0,
                                                   const int ubc_rows = 0)
{
    xi_o = NAN; aw_o = NAN; tol_o = INFINITY; it_o = 0;
    const int n = C.n;
    const double tlo = C.T[0], thi = C.T[n - 1];
    // ---------------- K crossing scans (optimal_buffer per group) ----------------
    bool all_eq = true;
#pragma unroll
    for (int k = 0; k < K; k++) {
        const double* __restrict__ Hk = C.H + (size_t)k * C.cap;
        bool any = false, all = true, prev = false;
        int fa = -1, la = -1, cin = -1, cout = -1;
        if (C.hsum) {
            struct { const double* hmax; const double* hmin; } S{C.hsum + (size_t)k * C.nblk,
                                                                 C.hsum + (size_t)(K + k) * C.nblk};
            buffer_scan_blocked(Hk, S, C.ntau, u, any, all, fa, la, cin, cout);
        } else {
            for (int i = 0; i < C.ntau; i++) {
                const bool ab = Hk[i] > u;
                any |= ab;
                all &= ab;
                if (ab) { if (fa < 0) fa = i; la = i; }
                if (i > 0) {
                    if (!prev && ab && cin < 0) cin = i - 1;
                    if (prev && !ab) cout = i - 1;
                }
                prev = ab;
            }
        }
        double a, b;
        if (!any) {
            a = C.T1; b = C.T1;
        } else if (all) {
            a = C.tau(0); b = C.tau(C.ntau - 1);
        } else {
            a = C.T1; b = C.T1;
            if (cin >= 0) {
                const double t0 = C.tau(cin), t1 = C.tau(cin + 1), h0 = Hk[cin], h1 = Hk[cin + 1];
                a = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
            }
            if (cout >= 0) {
                const double t0 = C.tau(cout), t1 = C.tau(cout + 1), h0 = Hk[cout], h1 = Hk[cout + 1];
                b = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
            }
            if (a == C.T1) a = C.tau(fa);
            if (b == C.T1) b = C.tau(la);
        }
        tin[k] = a;
        tout[k] = b;
        all_eq = all_eq && (a == b);
    }
    // the buffers are final here: store them now, so that they need no registers through the
    // validity check and the AW phase (only min(τ_k, ξ) is live there)
    if (tin_g)
#pragma unroll
        for (int k = 0; k < K; k++) tin_g[k] = tin[k];
    if (tout_g)
#pragma unroll
        for (int k = 0; k < K; k++) tout_g[k] = tout[k];
    if (all_eq) {
        st_o = SBR_NO_RUN_HR_BELOW_U | SBR_CONVERGED | lbits;
        tol_o = 0.0;
        return;
    }
    if (diag & 1) return; // timing diagnostics: stop after the crossing scans
    // ---------------- compute_ξ_hetero ----------------
    uint32_t flag = 0;
    double guess = (dist[0] * (tin[0] + tout[0])) / 2.0;
    double mo = tout[0];
#pragma unroll
    for (int k = 1; k < K; k++) { guess = guess + (dist[k] * (tin[k] + tout[k])) / 2.0; mo = dmax(mo, tout[k]); }
    double xmin = 0.0, xmax = mo * 2.0, xnew = guess;
    // exact brackets and values of the constant lookup points tin_k, tout_k
    int jin[K], jout[K];
    double gin[K], gout[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        jin[k] = -1; jout[k] = -1; gin[k] = 0.0; gout[k] = 0.0;
        if (tin[k] >= tlo && tin[k] <= thi) { jin[k] = ssl_range(C.T, 0, n - 1, tin[k]); gin[k] = C.lerp(jin[k], k, tin[k]); }
        if (tout[k] >= tlo && tout[k] <= thi) { jout[k] = ssl_range(C.T, 0, n - 1, tout[k]); gout[k] = C.lerp(jout[k], k, tout[k]); }
    }
    int jlo = 0, jhi = n - 1;
    uint32_t s = SBR_NO_RUN_MAXITER;
    double xi = NAN, tolr = INFINITY;
    bool term = false;
    double xt = 0.0, et = 0.0, awt = 0.0, errt = 0.0;
    int jt = 0;
    for (int iter = 1; iter <= max_iters; iter++) {
        it_o = iter;
        const double dd = xmin - xmax;
        if (collapsed(dd)) { s = SBR_NO_RUN_COLLAPSE; break; }
        if (iter == max_iters - 1) { s = SBR_NO_RUN_MAXITER; break; }
        const double xo = xnew;
        if (!(xo >= tlo)) { flag |= SBR_OOB; break; }  // searchsortedlast = 0: BoundsError
        const int j = ssl_range(C.T, jlo, jhi, xo); // t[jlo] <= ξmin <= xo <= ξmax < t[jhi+1]
        const int i2 = j + 1 < n - 1 ? j + 1 : n - 1;
        const double eps = C.T[i2] - C.T[j];
        double AW = 0.0;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double ic = dmin(tin[k], xo), oc = dmin(tout[k], xo);
            // value and bracket of oc, ic (each is either xo or the group constant)
            int joc, jic;
            double Goc, Gic;
            if (oc == xo) { joc = xo <= thi ? j : -1; Goc = joc >= 0 ? C.lerp(j, k, xo) : 0.0; }
            else { joc = jout[k]; Goc = gout[k]; }
            if (ic == xo) { jic = xo <= thi ? j : -1; Gic = jic >= 0 ? C.lerp(j, k, xo) : 0.0; }
            else { jic = jin[k]; Gic = gin[k]; }
            if (joc < 0 || jic < 0) flag |= SBR_OOB;
            // the slope probe only decides the terminal iterate: range checks every
            // iterate (BoundsError order of heterogeneity_solver.jl:81-95), lerps later
            const double xoe = oc + eps, xie = ic + eps;
            if (!(xoe <= thi && joc >= 0)) flag |= SBR_OOB;
            if (!(xie <= thi && jic >= 0)) flag |= SBR_OOB;
            AW = AW + dist[k] * (Goc - Gic);
        }
        if (flag) break;
        const double err = AW - kappa;
        if (fabs(err) <= tolerance) {
            // the terminal iterate: its slope probe runs after the loop, where the bracket state and
            // the constant lookups are dead (inside the loop it spilled them to scratch)
            term = true;
            xt = xo;
            jt = j;
            et = eps;
            awt = AW;
            errt = err;
            break;
        } else if (err > 0) {
            xmax = xo;
            jhi = j;
            xnew = 0.5 * (xo + xmin);
        } else {
            xmin = xo;
            jlo = j;
            xnew = 0.5 * (xo + xmax);
        }
    }
    if (flag) { st_o = flag | lbits; return; }
    if (term) {
        double AWe = 0.0;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double ic = dmin(tin[k], xt), oc = dmin(tout[k], xt);
            const int joc = oc == xt ? jt : jout[k], jic = ic == xt ? jt : jin[k];
            const double xoe = oc + et, xie = ic + et;
            const double Goce = C.lerp(ssl_gallop(C.T, n, joc, xoe), k, xoe);
            const double Gice = C.lerp(ssl_gallop(C.T, n, jic, xie), k, xie);
            AWe = AWe + dist[k] * (Goce - Gice);
        }
        if (AWe >= awt) { s = SBR_RUN; xi = xt; tolr = fabs(errt); }
        else s = SBR_FALSE_EQ;
    }
    if (s != SBR_RUN) { st_o = s | lbits; return; }
    if (diag & 2) return; // ... after the bisection

    // ---------------- is_valid_equilibrium_hetero ----------------
    // valid ⇔ no knot pair (t_{i−1}, t_i), t_i ≤ ξ, with AW(t_{i−1}) > κ ≥ AW(t_i), where
    // AW(t) = Σ dist_k (G_k(t) − G_k(max(0, t − τ_I,k))) (heterogeneity_solver.jl:190-207).
    {
        double tI[K];
        int jp[K];
#pragma unroll
        for (int k = 0; k < K; k++) { tI[k] = dmax(0.0, xi - tin[k]); jp[k] = 0; }
        bool prev = false, valid = true;
        // the reference's per-knot test on knots [i0, i1) with walkers jp at x(t_i0)'s bracket
        auto exact = [&](int i0, int i1) {
            for (int i = i0; i < i1; i++) {
                const double ti = C.T[i];
                double aw = 0.0;
#pragma unroll
                for (int k = 0; k < K; k++) {
                    const double a = C.lerp(i, k, ti);
                    const double x = dmax(0.0, ti - tI[k]);
                    while (jp[k] + 1 < n && C.T[jp[k] + 1] <= x) jp[k]++;
                    const double bb = C.lerp(jp[k], k, x);
                    aw = aw + dist[k] * (a - bb);
                }
                const bool above = aw > kappa;
                if (i > 0 && prev && !above) { valid = false; return; }
                prev = above;
            }
        };
        const int m = ssl_range(C.T, 0, n - 1, xi) + 1; // knots with t ≤ ξ (ξ ≥ t_0 here)
        if (!mono) {
            exact(0, m);
        } else {
            // 64-knot blocks bounded as in AW_max (G_k nondecreasing up to Δ_k): a block whose
            // bounds put every knot on one side of κ is decided without evaluating it; only
            // blocks straddling κ (near the crossing) are evaluated knot by knot.
            int hl[K], hh[K];
#pragma unroll
            for (int k = 0; k < K; k++) { hl[k] = 0; hh[k] = 0; }
            for (int i0 = 0; i0 < m && valid; i0 += 64) {
                const int i1 = (i0 + 64 < m ? i0 + 64 : m) - 1;
                double lb = 0.0, ub = 0.0;
#pragma unroll
                for (int k = 0; k < K; k++) {
                    // hints: the previous block's last bracket, then this block's first + its width
                    hl[k] = ssl_near(C.T, n, hh[k], dmax(0.0, C.T[i0] - tI[k]));
                    hh[k] = ssl_near(C.T, n, hl[k] + (i1 - i0), dmax(0.0, C.T[i1] - tI[k]));
                    const int kh = hh[k] + 1 < n - 1 ? hh[k] + 1 : n - 1;
                    lb = lb + dist[k] * (C.g(i0, k) - C.g(kh, k));
                    ub = ub + dist[k] * (C.g(i1, k) - C.g(hl[k], k));
                }
                lb = (lb - env) - 1e-14;
                ub = (ub + env) + 1e-14;
                if (ub <= kappa) {        // every knot not above κ
                    if (i0 > 0 && prev) valid = false;
                    prev = false;
                } else if (lb > kappa) {  // every knot above κ
                    prev = true;
                } else {
#pragma unroll
                    for (int k = 0; k < K; k++) jp[k] = hl[k];
                    exact(i0, i1 + 1);
                }
            }
        }
        if (!valid) { st_o = SBR_HETERO_INVALID | lbits; return; }
    }
    if (diag & 4) return; // ... after the validity check
    // ---------------- AW_max over the whole learning grid ----------------
    double icc[K], occ[K];
#pragma unroll
    for (int k = 0; k < K; k++) { icc[k] = dmin(tin[k], xi); occ[k] = dmin(tout[k], xi); }
    double mx = -INFINITY;
    // exact AW_total(t_i) for i in [i0, i1), walkers started by searches from per-group hints
    int ha[K], hb[K];
#pragma unroll
    for (int k = 0; k < K; k++) { ha[k] = 0; hb[k] = 0; }
    // the knot index each hint set was found for: a later search for knot i starts from
    // hint + (i − that index) (the shifted arguments move with the knots), not from the hint
    int ia = 0, ib = 0;
    auto eval_range = [&](int i0, int i1) {
        int ja[K], jb[K];
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double av = (C.T[i0] - xi) + icc[k], bv = (C.T[i0] - xi) + occ[k];
            ha[k] = ssl_near(C.T, n, ha[k] + (i0 - ia), av > 0 ? av : 0.0);
            hb[k] = ssl_near(C.T, n, hb[k] + (i0 - ib), bv > 0 ? bv : 0.0);
            ja[k] = ha[k];
            jb[k] = hb[k];
        }
        ia = i0;
        ib = i0;
        for (int i = i0; i < i1; i++) {
            const double ti = C.T[i];
            double cum = 0.0;
            // Interpolation weights shared between groups: groups with the same shift
            // (occ_k = ξ for most, equal icc_k where τ_IN,k ≥ ξ) have the same argument, bracket and
            // weight δ, so δ is divided out once; and a b argument on a knot (t_i − ξ + ξ == t_i)
            // has δ = 0 exactly — the same operands and operations as C.lerp, fewer divisions
            double xa_p = NAN, da_p = 0.0, xb_p = NAN, db_p = 0.0;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const double av = (ti - xi) + icc[k];
                const double bv = (ti - xi) + occ[k];
                const double xa = av > 0 ? av : 0.0;
                const double xb = bv > 0 ? bv : 0.0;
                if (!(xa <= thi) || !(xb <= thi)) flag |= SBR_OOB;
                while (ja[k] + 1 < n && C.T[ja[k] + 1] <= xa) ja[k]++;
                while (jb[k] + 1 < n && C.T[jb[k] + 1] <= xb) jb[k]++;
                const int qa = ja[k] > n - 2 ? n - 2 : (ja[k] < 0 ? 0 : ja[k]);
                const int qb = jb[k] > n - 2 ? n - 2 : (jb[k] < 0 ? 0 : jb[k]);
                double da = da_p, db = db_p;
                if (!(xa == xa_p)) da = (xa - C.T[qa]) / (C.T[qa + 1] - C.T[qa]);
                if (!(xb == xb_p)) {
                    const double t0 = C.T[qb], t1 = C.T[qb + 1];
                    db = (xb == t0 && t1 > t0) ? 0.0 : (xb - t0) / (t1 - t0);
                }
                xa_p = xa; da_p = da; xb_p = xb; db_p = db;
                const double gi = C.g(qa, k) * (1.0 - da) + C.g(qa + 1, k) * da;
                const double go = C.g(qb, k) * (1.0 - db) + C.g(qb + 1, k) * db;
                const double awin = av >= 0 ? gi : 0.0;
                const double awout = bv >= 0 ? go : 0.0;
                cum = cum + dist[k] * (awout - awin);
            }
            if (aw_path) aw_path[i] = cum;
            if (mx == mx && (cum != cum || cum > mx)) mx = cum;
        }
    };
    if (!mono) {
        eval_range(0, n);
    } else {
        // Every group CDF is nondecreasing on the knots up to its drawdown Δ_k, so over knots
        // [i0, i1] AW_OUT,k is at most G_k at the knot after b_k(t_i1)'s bracket + Δ_k and AW_IN,k
        // at least G_k at a_k(t_i0)'s bracket − Δ_k (0 where masked; `env` = Σ dist_k·2Δ_k):
        // branch and bound over 256/64/8-knot ranges,
        // the same maximum with a fraction of the K·2 lerps per knot.  Arguments are
        // nondecreasing in i, so the last knot's range check covers the whole path.
#pragma unroll
        for (int k = 0; k < K; k++) {
            const double av = (C.T[n - 1] - xi) + icc[k], bv = (C.T[n - 1] - xi) + occ[k];
            if (!((av > 0 ? av : 0.0) <= thi) || !((bv > 0 ? bv : 0.0) <= thi)) flag |= SBR_OOB;
        }
        auto ub_rng = [&](int i0, int i1) -> double {
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const double bv = (C.T[i1] - xi) + occ[k];
                double hi = 0.0;
                if (sep && occ[k] == xi) {
                    // b_k(t_i1) = (t_i1 − ξ) + ξ lies within an ulp of t_i1, below t[i1 + koff] (knots
                    // koff apart are farther apart than that, `sep`): G_k at the knot after its
                    // bracket is G_k at a knot <= i1 + koff, no search
                    const double g = C.g(i1 + koff < n - 1 ? i1 + koff : n - 1, k);
                    hi = g > 0.0 ? g : 0.0;
                    hb[k] = i1; // with ib = i1 below, the next hint hb + (i − ib) is i itself
                } else if (bv >= 0) {
                    hb[k] = ssl_near(C.T, n, hb[k] + (i1 - ib), bv);
                    const double g = C.g(hb[k] + 1 < n - 1 ? hb[k] + 1 : n - 1, k);
                    hi = g > 0.0 ? g : 0.0;
                }
                const double av = (C.T[i0] - xi) + icc[k];
                double lo = 0.0;
                if (av >= 0) {
                    ha[k] = ssl_near(C.T, n, ha[k] + (i0 - ia), av);
                    lo = C.g(ha[k], k);
                } else {
                    lo = C.g(0, k) < 0.0 ? C.g(0, k) : 0.0;
                }
                sum = sum + dist[k] * (hi - lo);
            }
            ia = i0;
            ib = i1;
            return (sum + 1e-14) + env;
        };
        auto end_of = [&](int i0, int w) { return i0 + w < n ? i0 + w : n; };
        if (!flag) {
            // pass 1 keeps every range bound as a code in LDS (this lane's column of ubc rows:
            // the 256-knot ranges, then the best one's four 64-knot and its eight 8-knot ranges),
            // c = ceil(S·ub) clamped to [0, S − 2] — c/S >= ub exactly (S = 2^bits: ×S is exact) —
            // or S − 1 (ub > (S − 2)/S: unknown).  Pass 2: c/S <= mx prunes, (c − 1)/S >= mx
            // descends (ub > mx), in between — and for rows past ubc_rows, the LDS left — the bound
            // is recomputed (ub_rng's value does not depend on the hints).
            constexpr double S = (double)(1 << kHetUbcBits), rS = 1.0 / S;
            constexpr int unk = (1 << kHetUbcBits) - 1;
            const int nr = (n + 255) >> 8;
            auto put = [&](int row, double ub) {
                if (row >= ubc_rows) return;
                const double q = ceil(ub * S);
                ubc[row * ubc_stride] = (ubc_t)(q != q || q > S - 2.0 ? unk : (q < 0.0 ? 0 : (int)q));
            };
            auto pruned = [&](int row, int i0, int i1) -> bool {
                if (row < ubc_rows) {
                    const int cv = ubc[row * ubc_stride];
                    if (cv != unk) {
                        if ((double)cv * rS <= mx) return true;
                        if ((double)(cv - 1) * rS >= mx) return false;
                    }
                }
                return ub_rng(i0, i1) <= mx;
            };
            int bs = 0;
            double bu = -INFINITY;
            for (int i0 = 0; i0 < n; i0 += 256) {
                const double ub = ub_rng(i0, end_of(i0, 256) - 1);
                put(i0 >> 8, ub);
                if (!(ub <= bu)) { bu = ub; bs = i0; }
            }
            int bb = bs;
            bu = -INFINITY;
            for (int i0 = bs; i0 < end_of(bs, 256); i0 += 64) {
                const double ub = ub_rng(i0, end_of(i0, 64) - 1);
                put(nr + ((i0 - bs) >> 6), ub);
                if (!(ub <= bu)) { bu = ub; bb = i0; }
            }
            int b8 = bb;
            bu = -INFINITY;
            for (int i0 = bb; i0 < end_of(bb, 64); i0 += 8) {
                const double ub = ub_rng(i0, end_of(i0, 8) - 1);
                put(nr + 4 + ((i0 - bb) >> 3), ub);
                if (!(ub <= bu)) { bu = ub; b8 = i0; }
            }
            eval_range(b8, end_of(b8, 8));
            for (int s0 = 0; s0 < n && mx == mx; s0 += 256) {
                const int se = end_of(s0, 256);
                if (pruned(s0 >> 8, s0, se - 1)) continue;
                for (int k0 = s0; k0 < se && mx == mx; k0 += 64) {
                    const int ke = end_of(k0, 64);
                    if (s0 == bs ? pruned(nr + ((k0 - bs) >> 6), k0, ke - 1) : (ub_rng(k0, ke - 1) <= mx)) continue;
                    for (int i0 = k0; i0 < ke && mx == mx; i0 += 8) {
                        const int ie = end_of(i0, 8);
                        if (i0 == b8) continue;
                        if (k0 == bb ? pruned(nr + 4 + ((i0 - bb) >> 3), i0, ie - 1) : (ub_rng(i0, ie - 1) <= mx))
                            continue;
                        eval_range(i0, ie);
                    }
                }
            }
        }
    }
    if (flag) { st_o = flag | lbits; return; }
    xi_o = xi;
    tol_o = tolr;
    aw_o = mx;
    st_o = SBR_RUN | SBR_CONVERGED | lbits;
}

constexpr int kHetBlock = 256; // u points per hetero equilibrium workgroup (512 was slower)
constexpr int kHetMinW = 2; // waves per SIMD: two 4-wave workgroups per CU (LDS slab: kHetLds in sbr_capi.hip)
template <int K, int BLOCK, int MODE>
__global__ __launch_bounds__(BLOCK, kHetMinW)
void equilibrium_hetero_kernel(HeteroBufs L, const double* __restrict__ dist,
                                                                   const double* __restrict__ eta,
                                                                   const double* __restrict__ t_end,
                                                                   const double* __restrict__ u, HeteroEqArgs a,
                                                                   ResultSoA out, double* __restrict__ tin_out,
                                                                   double* __restrict__ tout_out)
{
    extern __shared__ double smem[];
    __builtin_amdgcn_s_setprio(2); // issue priority over co-resident learning waves (step 49.7 -> 47.9 ms)
    // XCD-aware tile order (1-D grid): workgroup w runs on XCD w mod 8, so the u-tiles of one
    // column are given to consecutive workgroups of the same XCD — they share that XCD's L2
    // copy of the column's G and HR rows instead of fetching four copies into four L2s.
    const int ntile = (a.n_u + BLOCK - 1) / BLOCK;
    const int wid = blockIdx.x, xcd = wid & 7, seq = wid >> 3;
    const int c = (seq / ntile) * 8 + xcd;
    const int tile = seq - (seq / ntile) * ntile;
    if (c >= a.n_col) return;
    const int n = L.n_knots[c];
    const uint32_t lst = L.status[c];
    const size_t cap = (size_t)L.cap;
    const double* __restrict__ gT = L.t + (size_t)c * cap;
    const bool fits = n <= a.lds_cap;
    // MODE 1: columns whose knot times fit the LDS slab; MODE 2: the others (global-memory path,
    // launched second without a slab); the hot launch carries one copy of the point solve
    if ((MODE == 1 && !fits) || (MODE == 2 && fits)) return;
    __shared__ int s_nonmono;
    __shared__ int s_close; // two knots 2 apart closer than 1e-15·t[n−1] (the AW bounds then search)
    __shared__ int s_close1; // two consecutive knots that close (the AW bounds then use knot + 2)
    if (threadIdx.x == 0) { s_nonmono = a.exhaustive || a.aw_path; s_close = 0; s_close1 = 0; } // path mode: every knot
    if (fits)
        for (int i = threadIdx.x; i < n; i += BLOCK) smem[i] = gT[i];
    __syncthreads();

    // Group CDF drawdown for the AW_max branch and bound: Tsit5 at eps() leaves ulp-sized
    // decreases in the saturated tail (G_k = 1 − 2^-53 after 1.0: most config-4 columns), so
    // the bounds take G_k[j] ± Δ_k for the prefix max / suffix min, with
    // Δ_k = (#decreases)·(largest decrease) ≥ the largest drawdown max_{j<j'} G_k[j] − G_k[j'].
    // NaN or ±Inf anywhere -> exhaustive evaluation.
    __shared__ int s_dcnt[K];
    __shared__ unsigned long long s_dmax[K];
    if (threadIdx.x < K) { s_dcnt[threadIdx.x] = 0; s_dmax[threadIdx.x] = 0ull; }
    __syncthreads();
    {
        const double* __restrict__ Gc = L.G + (size_t)c * cap * K;
        bool nan = false;
        int cnt[K];
        double dm[K];
#pragma unroll
        for (int k = 0; k < K; k++) { cnt[k] = 0; dm[k] = 0.0; }
        for (int i = 1 + threadIdx.x; i < n; i += BLOCK)
#pragma unroll
            for (int k = 0; k < K; k++) {
                const double g1 = Gc[(size_t)i * K + k], g0 = Gc[(size_t)(i - 1) * K + k];
                if (!(fabs(g0) < INFINITY) || !(fabs(g1) < INFINITY)) nan = true; // NaN or ±Inf
                else if (g1 < g0) { cnt[k]++; dm[k] = dmax(dm[k], g0 - g1); }
            }
        if (nan) s_nonmono = 1;
        if (fits) {
            bool close = false, close1 = false;
            const double sepd = n > 0 ? 1e-15 * smem[n - 1] : 0.0; // n == 0: an ARG_INVALID column
            for (int i = threadIdx.x; i + 2 < n; i += BLOCK) close |= !(smem[i + 2] - smem[i] > sepd);
            for (int i = threadIdx.x; i + 1 < n; i += BLOCK) close1 |= !(smem[i + 1] - smem[i] > sepd);
            if (close) s_close = 1;
            if (close1) s_close1 = 1;
        }
#pragma unroll
        for (int k = 0; k < K; k++)
            if (cnt[k]) {
                atomicAdd(&s_dcnt[k], cnt[k]);
                atomicMax(&s_dmax[k], (unsigned long long)__double_as_longlong(dm[k])); // dm > 0: ordered as bits
            }
    }
    // per-group 64-entry block max / min of HR (sbr_scan.h) at the top of the LDS slab
    const int ntau = L.n_tau[c];
    const int nblk = (ntau + 63) >> 6;
    const bool sums = fits && n + 2 * K * nblk <= a.lds_cap;
    double* hsum = smem + (a.lds_cap - 2 * K * nblk);
    if (sums) {
        const double* __restrict__ Hc = L.hr + (size_t)c * K * cap;
        for (int q = threadIdx.x; q < K * nblk; q += BLOCK) {
            const int k = q / nblk, bk = q - k * nblk;
            const double* __restrict__ Hk = Hc + (size_t)k * cap;
            double mx = -INFINITY, mn = INFINITY;
            const int e = (bk << 6) + 64 < ntau ? (bk << 6) + 64 : ntau;
            for (int i = bk << 6; i < e; i++) {
                const double h = Hk[i];
                if (h > mx) mx = h;                            // NaN never > u: ignore it
                mn = (h != h) ? -INFINITY : (h < mn ? h : mn);  // NaN is "not above"
            }
            hsum[(size_t)k * nblk + bk] = mx;
            hsum[(size_t)(K + k) * nblk + bk] = mn;
        }
    }
    __syncthreads();
    const bool mono = s_nonmono == 0;
    double env = 0.0; // Σ_k dist_k · 2Δ_k, added to every branch-and-bound bound
#pragma unroll
    for (int k = 0; k < K; k++)
        env = env + dist[k] * (2.0 * ((double)s_dcnt[k] * __longlong_as_double((long long)s_dmax[k])));
    const int j = tile * BLOCK + threadIdx.x;
    if (j >= a.n_u) return;
    double dl[K];
#pragma unroll
    for (int k = 0; k < K; k++) dl[k] = dist[k];
    const double uj = u[j];
    const uint32_t lbits = lst & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED | SBR_KNOT_OVERFLOW);
    double xi, aw, tol, tin[K], tout[K];
    uint32_t st;
    int it;
    const size_t o = (size_t)c * (size_t)a.n_u + j;
    double* const tin_g = tin_out ? tin_out + o * K : nullptr;
    double* const tout_g = tout_out ? tout_out + o * K : nullptr;
    if ((lst & (SBR_ARG_INVALID | SBR_OOB)) || n < 2 || !(uj >= 0.0)) {
        xi = NAN; aw = NAN; tol = INFINITY; it = 0;
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (tin_g) tin_g[k] = NAN;
            if (tout_g) tout_g[k] = NAN;
        }
        st = ((lst & SBR_ARG_INVALID) || !(uj >= 0.0)) ? SBR_ARG_INVALID : (SBR_OOB | lbits);
    } else if constexpr (MODE == 1) {
        HCol<K, const double*> C{smem, L.G + (size_t)c * cap * K, L.hr + (size_t)c * K * cap, n, L.n_tau[c],
                                 L.n_le[c], cap, eta[c], t_end[c], sums && !a.exhaustive ? hsum : nullptr, nblk};
        // AW_max's byte bound cache: rows of BLOCK bytes (one per lane) between the knot times
        // and the HR block sums
        const int ubc_rows = ((sums ? a.lds_cap - 2 * K * nblk : a.lds_cap) - n) * 8 / (BLOCK * (int)sizeof(ubc_t));
        ubc_t* const ubc = (ubc_t*)(smem + n) + threadIdx.x;
        solve_hetero_point<K>(C, dl, uj, a.kappa, a.max_iters, a.tolerance, lbits, xi, aw, tol, st, it, tin, tout,
                              mono, a.diag, a.aw_path, env, fits && s_close == 0, s_close1 == 0 ? 1 : 2,
                              tin_g, tout_g, ubc, BLOCK, ubc_rows);
    } else {
        HCol<K, const double*> C{gT, L.G + (size_t)c * cap * K, L.hr + (size_t)c * K * cap, n, L.n_tau[c],
                                 L.n_le[c], cap, eta[c], t_end[c], nullptr, 0};
        solve_hetero_point<K>(C, dl, uj, a.kappa, a.max_iters, a.tolerance, lbits, xi, aw, tol, st, it, tin, tout,
                              mono, a.diag, a.aw_path, env, fits && s_close == 0, s_close1 == 0 ? 1 : 2,
                              tin_g, tout_g);
    }
    out.xi[o] = xi;
    out.aw_max[o] = aw;
    out.tol[o] = tol;
    out.status[o] = st;
    if (out.iters) out.iters[o] = it;
}

template <int K>
static hipError_t launch_hetero_k(const double* betas, const double* dist, const double* eta, const double* t_end,
                                  const double* u, const LearnArgs& la, const HeteroEqArgs& ea_in, const HeteroBufs& L,
                                  const ResultSoA& out, double* tin, double* tout, hipStream_t s, int phase)
{
    if (phase == 2) { // hazards of knots already in L (caller knots)
        hipLaunchKernelGGL(hazard_hetero_kernel<K>, dim3(la.n_beta), dim3(64), 0, s, betas, dist, eta, la, L);
        return hipGetLastError();
    }
    if (phase == 0) {
        hipLaunchKernelGGL(learn_hetero_wave_kernel<K>, dim3((la.n_beta + kHetLearnWG - 1) / kHetLearnWG),
                           dim3(64 * kHetLearnWG), 0, s, betas, dist, eta, t_end, la, L);
        return hipGetLastError();
    }
    const size_t lds = (size_t)ea_in.lds_cap * sizeof(double);
    HeteroEqArgs ea = ea_in;
    ea.n_col = la.n_beta;
    // the LDS-resident columns, then (no slab, exiting at once where the knots fit) the others
    auto go = [&](auto k1, auto k2, dim3 grid, int bs) {
        hipLaunchKernelGGL(k1, grid, dim3(bs), lds, s, L, dist, eta, t_end, u, ea, out, tin, tout);
        hipLaunchKernelGGL(k2, grid, dim3(bs), 0, s, L, dist, eta, t_end, u, ea, out, tin, tout);
    };
    const unsigned ncol8 = (unsigned)((la.n_beta + 7) / 8) * 8;
    if (ea.n_u >= kHetBlock)
        go(equilibrium_hetero_kernel<K, kHetBlock, 1>, equilibrium_hetero_kernel<K, kHetBlock, 2>,
           dim3(((ea.n_u + kHetBlock - 1) / kHetBlock) * ncol8), kHetBlock);
    else
        go(equilibrium_hetero_kernel<K, 64, 1>, equilibrium_hetero_kernel<K, 64, 2>, dim3(((ea.n_u + 63) / 64) * ncol8), 64);
    return hipGetLastError();
}

hipError_t launch_hetero(int K, const double* betas, const double* dist, const double* eta, const double* t_end,
                         const double* u, const LearnArgs& la, const HeteroEqArgs& ea, const HeteroBufs& L,
                         const ResultSoA& out, double* tin, double* tout, hipStream_t s, int phase)
{
    switch (K) {
    case 1: return launch_hetero_k<1>(betas, dist, eta, t_end, u, la, ea, L, out, tin, tout, s, phase);
    case 2: return launch_hetero_k<2>(betas, dist, eta, t_end, u, la, ea, L, out, tin, tout, s, phase);
    case 3: return launch_hetero_k<3>(betas, dist, eta, t_end, u, la, ea, L, out, tin, tout, s, phase);
    case 4: return launch_hetero_k<4>(betas, dist, eta, t_end, u, la, ea, L, out, tin, tout, s, phase);
    case 8: return launch_hetero_k<8>(betas, dist, eta, t_end, u, la, ea, L, out, tin, tout, s, phase);
    default: return hipErrorInvalidValue;
    }
}

// ---------------------------------------------------------------------------
// hetero_aw_groups_kernel<K>: get_AW_hetero's per-group curves (heterogeneity_solver.jl:335-362)
// of one solved point on its learning knots, one lane per knot i:
//   AW_OUT_k(t_i) = t_i − ξ + min(τ̄_OUT,k, ξ) >= 0 ? G_k(max(that, 0)) : 0, AW_IN_k alike,
// G_k the gridded-linear interpolant on the knots (bracket = searchsortedlast, clamped to
// [0, n−2]) — the operations of equilibrium_hetero_kernel's AW pass, so the same bits.  Runs
// after the equilibrium on the same stream (ξ, τ̄ and status read on the device); writes nothing
// without a run (the host fills NaN rows).  Rows: AW_OUT_k at out + k·ld, AW_IN_k at out + (K+k)·ld.
// ---------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256) void hetero_aw_groups_kernel(const double* __restrict__ T,
                                                               const double* __restrict__ G,
                                                               const int32_t* __restrict__ n_p,
                                                               const double* __restrict__ xi_p,
                                                               const double* __restrict__ tin,
                                                               const double* __restrict__ tout,
                                                               const uint32_t* __restrict__ status,
                                                               double* __restrict__ out, size_t ld)
{
    const int n = *n_p;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n || n < 2 || !(status[0] & SBR_RUN)) return;
    const double xi = *xi_p, ti = T[i];
    auto at = [&](int k, double x) {
        int q = ssl_range(T, 0, n - 1, x);
        q = q > n - 2 ? n - 2 : (q < 0 ? 0 : q);
        const double d = (x - T[q]) / (T[q + 1] - T[q]);
        return G[(size_t)q * K + k] * (1.0 - d) + G[(size_t)(q + 1) * K + k] * d;
    };
#pragma unroll
    for (int k = 0; k < K; k++) {
        const double av = (ti - xi) + dmin(tin[k], xi);
        const double bv = (ti - xi) + dmin(tout[k], xi);
        const double gi = at(k, av > 0 ? av : 0.0);
        const double go = at(k, bv > 0 ? bv : 0.0);
        out[(size_t)k * ld + i] = bv >= 0 ? go : 0.0;
        out[(size_t)(K + k) * ld + i] = av >= 0 ? gi : 0.0;
    }
}

hipError_t launch_hetero_aw_groups(int K, const double* T, const double* G, const int32_t* n_dev, int n_max,
                                   const double* xi, const double* tin, const double* tout, const uint32_t* status,
                                   double* out, size_t ld, hipStream_t s)
{
    if (n_max < 1) return hipSuccess;
    const dim3 grid((unsigned)((n_max + 255) / 256)), block(256);
    switch (K) {
    case 1: hipLaunchKernelGGL(hetero_aw_groups_kernel<1>, grid, block, 0, s, T, G, n_dev, xi, tin, tout, status, out, ld); break;
    case 2: hipLaunchKernelGGL(hetero_aw_groups_kernel<2>, grid, block, 0, s, T, G, n_dev, xi, tin, tout, status, out, ld); break;
    case 3: hipLaunchKernelGGL(hetero_aw_groups_kernel<3>, grid, block, 0, s, T, G, n_dev, xi, tin, tout, status, out, ld); break;
    case 4: hipLaunchKernelGGL(hetero_aw_groups_kernel<4>, grid, block, 0, s, T, G, n_dev, xi, tin, tout, status, out, ld); break;
    case 8: hipLaunchKernelGGL(hetero_aw_groups_kernel<8>, grid, block, 0, s, T, G, n_dev, xi, tin, tout, status, out, ld); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sbr
