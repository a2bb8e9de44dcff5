// sbr_baseline.hip — gfx950 kernels for the baseline β×u sweep.
//
//   learn_logistic_kernel   one lane per β column: FP64 Tsit5 with
//                           OrdinaryDiffEq's PI step control on
//                           dx/dt = βx(1−x) (learning.jl:41-54), every
//                           accepted step a knot (save_everystep), hazard
//                           numerator / cumulative trapezoid streamed as the
//                           knots are produced (solver.jl:153-185), HR
//                           finalised in a second pass.
//   equilibrium_kernel      one workgroup per (β, u-tile), one lane per grid
//                           point: knot grid + HR staged once per workgroup
//                           in LDS, then per lane the crossing scan
//                           (solver.jl:211-264), the ξ bisection with the
//                           slope check (solver.jl:308-376) and the AW path
//                           maximum (solver.jl:495-532, 565).  Results are
//                           written as coalesced SoA rows.
//
// Bit-exact against oracle/sbr_oracle.c (see sbr_device.h).
#include "sbr_device.h"
#include "sbr_kernels.h"
#include "sbr_ode.h"
#include "sbr_scan.h"

namespace sbr {

// ============================================================================
// Learning kernel
// ============================================================================
// lanes per learning workgroup of the pipelined batch's streamed-hazard launches (learning that
// runs beside the equilibrium kernel): two waves per workgroup.  Same-call A/Bs (r05_oo, r05_pp):
// the co-running equilibrium kernel 1.39 -> 1.36 ms, config-3 step 1.487-1.507 -> 1.455 ms at 50
// steps; 256 lanes slower (1.524 ms).  Latency-critical launches (single sweeps, the batch's
// first group, config 1) keep one wave per workgroup: with two, config 1 took 2.24 instead of
// 2.15 ms and a single sweep 4.20 instead of 4.01 ms (r05_qq)
constexpr int kLearnBlock = 128;
constexpr int kLearnBlockLat = 64;

// readiness sweeps: column b is complete (knots, counters, status written by this lane) —
// release it to the equilibrium workgroups (agent scope: they run on other CUs / XCDs)
__device__ __forceinline__ void publish_column(const LearnArgs& a, int b)
{
    const int k = atomicAdd(a.ready_tail, 1);
    __hip_atomic_store(a.ready_q + k, b + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
// one lane's knot-row store of the learning kernel (the nontemporal hint was neutral, r05_ee)
#define st_knot(p, v) (*(p) = (v))
// STAGE (a batch's wide learning launch, the chip otherwise idle; fused hazard): the knot rows
// (t, G) and the hazard rows (numerator, running integral) go through a per-lane ring of
// kStageSlots slots in LDS, [array][slot][lane], and leave as whole 128-B lines — eight 16-B
// stores per array — on every 8th attempted step (the same step for every live lane), the rest
// when the lane's solve ends.  With hundreds of learning waves the direct 8-B knot stores (one
// line per lane per store instruction) made the launch twice the chain alone
// (tools/ubench_wide.hip: 640 waves 3.74 ms without stores, 6.48 direct, 4.43 staged).  Between
// two flushes a lane accepts at most 8 knots and holds fewer than 16 unflushed after one, so 24
// slots never overwrite an unflushed entry; 48 KiB per wave lets three waves share a CU.
constexpr int kStageSlots = 24;
constexpr size_t kStageLdsPerWave = (size_t)4 * kStageSlots * 64 * sizeof(double); // 48 KiB
template <int LB, bool STAGE = false>
__global__ __launch_bounds__(LB) void learn_logistic_kernel(const double* __restrict__ beta,
                                                            const double* __restrict__ eta,
                                                            const double* __restrict__ t_end, LearnArgs a,
                                                            LearnBufs L)
{
    extern __shared__ double stage_lds[];
    // latency-bound (one serial ODE per lane): take issue priority over co-resident
    // equilibrium waves of a previous batch
    __builtin_amdgcn_s_setprio(3);
    // one column per lane (a knot store or load of the wave touches one row per active lane).
    // Heads first (a.wpg, one-wave blocks): the workgroup dispatcher deals consecutive blocks
    // round-robin over the XCDs and their CUs, so every grid's first wave — block g·32 of a
    // 2048-column grid — landed on one of only 8 CUs, three heads per CU, and those waves hold
    // the longest columns of a β-descending grid (config 3: column 22, 4.45k steps against a
    // 2.9k median).  Dealt first, each head has a CU to itself: a 20-grid launch 4.2-4.7 →
    // 3.0-3.2 ms (tools/ubench_fill.hip).
    int blk = blockIdx.x;
    if (LB == 64 && a.wpg) {
        const int nh = (a.n_beta / (64 * a.wpg)) * a.head, per = a.wpg - a.head;
        blk = blk < nh ? (blk / a.head) * a.wpg + blk % a.head
                       : ((blk - nh) / per) * a.wpg + a.head + (blk - nh) % per;
    }
    const int b = blk * LB + threadIdx.x;
    const bool live = b < a.n_beta;
    const double BETA = live ? beta[b] : 1.0, ETA = live ? eta[b] : 1.0, T1 = live ? t_end[b] : 1.0, T0 = 0.0;
    const size_t row = (size_t)(live ? b : 0) * (size_t)L.cap;
    double* __restrict__ T = L.t + row;
    double* __restrict__ Gv = L.G + row;
    uint32_t st = 0;
    const bool fuse = a.fuse_hazard != 0; // wave-uniform

    if (live && (!(BETA > 0.0) || !(T1 > T0) || !(ETA > 0.0))) { // LearningParameters / EconomicParameters checks
        L.status[b] = SBR_ARG_INVALID;
        L.n_knots[b] = 0; L.n_tau[b] = 0; L.n_le[b] = 0; L.n_accept[b] = 0; L.n_reject[b] = 0;
        if (a.ready_q) publish_column(a, b);
    } else if (live) {
    // ---- knot sink: store (t, G).  Branch-free: every attempted step writes its candidate
    // knot at the fill index n (a rejected one is overwritten by the next accepted step) and the
    // counters advance by select.  Fused hazard (a.fuse_hazard, the pipelined batch): each
    // accepted knot ≤ η is also a τ̄ entry of hazard_rate (solver.jl:153-185) — its numerator
    // (p·e^{λτ̄})·g and the running trapezoid integral I are formed as the knot is accepted
    // (g = βG(1−G), the sequential sum in the reference's order), the η entry at the first
    // knot past η; the normalisation by p·I + (1−p)·I_η is hazard_norm_kernel's.  The same
    // operations as hazard_kernel, so the same bits. ----
    struct Sink {
        double* __restrict__ T;
        double* __restrict__ Gv;
        double* __restrict__ H;
        double* __restrict__ HI;
        double* SL;       // STAGE: this lane's ring, slot k of array a at SL[(a·kStageSlots + k)·64]
        int fl, tick;     // STAGE: entries flushed (a multiple of 16), attempted steps
        int ws, fs;       // STAGE: the ring slots of entry n and of entry fl
        int n, cap, m; // m: knots ≤ η (the hazard stage's τ̄ prefix), set at the first knot past η
        double tlast, bound, eta;
        int past, done, stop_after_eta; // 0 / 1 (ints: loop-carried bools cost mask conversions)
        uint32_t& st;
        int fuse, hm;            // hm: τ̄ entries written
        double beta, lam, p;
        double hI, he, ht, hg;   // I, e and τ̄ of the last τ̄ entry, pdf of the last knot ≤ η
        __device__ __forceinline__ bool push(bool acc, double t, double x)
        {
            const bool room = n < cap;
            const int w = room ? n : cap - 1;
            if (STAGE) {
                if (room) { SL[ws * 64] = t; SL[(kStageSlots + ws) * 64] = x; }
            } else if (room) {
                st_knot(T + w, t); st_knot(Gv + w, x); // a rejected candidate is overwritten later
            }
            // bitwise (not short-circuit) logic: selects, no branches
            const bool pushed = acc & room;
            const bool over = acc & !room;
            st |= over ? SBR_KNOT_OVERFLOW : 0u;
            // furthest point any lookup of the equilibrium stage can reach (DESIGN.md
            // §Truncation): max of t_j + (t_j − t_{j−1}) over the knots j ≥ 1 up to and
            // including the first knot past η
            const bool upd = pushed & (n >= 1) & (past == 0);
            const double reach = dmax(bound, t + (t - tlast));
            bound = upd ? reach : bound;
            const bool cross = pushed & (past == 0) & (t > eta);
            if (fuse) {
                const double g = (beta * x) * (1.0 - x);
                const bool le = pushed & (past == 0) & (t <= eta);
                const double E = sbr_exp(lam * t);
                const double e = E * g;
                const double In = hm == 0 ? 0.0 : hI + (0.5 * (he + e)) * (t - ht);
                if (STAGE) {
                    if (le) { SL[(2 * kStageSlots + ws) * 64] = (p * E) * g; SL[(3 * kStageSlots + ws) * 64] = In; }
                } else if (le) {
                    st_knot(H + n, (p * E) * g); st_knot(HI + n, In);
                }
                hI = le ? In : hI;
                he = le ? e : he;
                ht = le ? t : ht;
                hg = le ? g : hg;
                hm += le ? 1 : 0;
                if (cross && ht != eta) {
                    // τ̄ = η on bracket [m-1, m]: pdf interpolated, pushed unless η is a knot
                    const double d = (eta - ht) / (t - ht);
                    const double pe = hg * (1.0 - d) + g * d;
                    const double E2 = sbr_exp(lam * eta);
                    const double e2 = E2 * pe;
                    hI = hI + (0.5 * (he + e2)) * (eta - ht);
                    if (STAGE) { // hm == n here: every earlier knot is ≤ η
                        SL[(2 * kStageSlots + ws) * 64] = (p * E2) * pe;
                        SL[(3 * kStageSlots + ws) * 64] = hI;
                    } else {
                        H[hm] = (p * E2) * pe;
                        HI[hm] = hI;
                    }
                    hm++;
                }
            }
            m = cross ? n : m;
            past |= cross ? 1 : 0;
            tlast = pushed ? t : tlast;
            n += pushed ? 1 : 0;
            if (STAGE) {
                ws = pushed ? (ws == kStageSlots - 1 ? 0 : ws + 1) : ws;
                if ((++tick & 7) == 0 && n - fl >= 16) flush_line();
            }
            done |= (over | (pushed & (stop_after_eta != 0) & (past != 0) & (t >= bound))) ? 1 : 0;
            return done == 0;
        }
        // STAGE: entries [fl, fl + 16) from the ring to the rows, as 16-B pairs (hazard entries
        // past the τ̄ grid carry stale slots: never read)
        __device__ __forceinline__ void flush_line()
        {
            typedef double d2 __attribute__((ext_vector_type(2)));
            double* const R[4] = {T, Gv, H, HI};
#pragma unroll
            for (int k = 0; k < 16; k += 2) {
                const int s0 = fs + k < kStageSlots ? fs + k : fs + k - kStageSlots; // pairs never straddle the wrap
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    d2 v;
                    v.x = SL[(q * kStageSlots + s0) * 64];
                    v.y = SL[(q * kStageSlots + s0 + 1) * 64];
                    *(d2*)(R[q] + fl + k) = v;
                }
            }
            fl += 16;
            fs = fs + 16 < kStageSlots ? fs + 16 : fs + 16 - kStageSlots;
        }
        __device__ __forceinline__ bool start(double t, double x) { return push(true, t, x); }
        __device__ __forceinline__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&, bool)
        {
            return push(acc, tn, y1);
        }
        // the column is learned: counters and status, then (readiness sweeps) its
        // publication — called by ode_scalar the moment this lane's solve ends, while the
        // other columns of the wave may still be integrating
        const LearnBufs* Lp;
        const LearnArgs* ap;
        int b;
        int ntau_out; // the τ̄ entries of the column, set by finish
        __device__ __forceinline__ void finish(const OdeOut& o)
        {
            if (STAGE) // the entries not flushed yet: knots [fl, n), τ̄ entries [fl, hm)
                for (int i = fl, sl = fs; i < n; i++, sl = sl == kStageSlots - 1 ? 0 : sl + 1) {
                    T[i] = SL[sl * 64];
                    Gv[i] = SL[(kStageSlots + sl) * 64];
                    if (i < hm) {
                        H[i] = SL[(2 * kStageSlots + sl) * 64];
                        HI[i] = SL[(3 * kStageSlots + sl) * 64];
                    }
                }
            st |= o.status;
            int n_le = m < 0 ? n : m; // every knot ≤ η when none passed it
            int n_tau = 0;
            if (fuse) {
                // hazard_kernel's η rule: with no knot past η, pdf(η) exists only if η is the last knot
                if (m < 0 && ht != eta) {
                    st |= SBR_OOB;
                    n_le = 0;
                } else {
                    n_tau = hm;
                }
            }
            Lp->n_knots[b] = n;
            Lp->n_le[b] = n_le;
            if (fuse) Lp->n_tau[b] = n_tau;
            ntau_out = n_tau;
            Lp->status[b] = st;
            Lp->n_accept[b] = (int)o.naccept;
            Lp->n_reject[b] = (int)o.nreject;
            if (ap->ready_q) publish_column(*ap, b);
        }
    } sink{T, Gv, fuse ? L.hr + row : nullptr, fuse ? L.hrI + row : nullptr,
           stage_lds + (size_t)(threadIdx.x >> 6) * (4 * kStageSlots * 64) + (threadIdx.x & 63), 0, 0, 0, 0,
           0, L.lim, -1, 0.0, -INFINITY, ETA,
           0, 0, a.stop_after_eta != 0 ? 1 : 0, st, fuse ? 1 : 0, 0, BETA, a.lam, a.p, 0.0, 0.0, 0.0, 0.0,
           &L, &a, b, 0};
    LogisticSys f{BETA};
    OdeOut o;
    ode_scalar(f, sink, T1, a.x0, a.rtol, a.atol, a.maxiters, o);
    if (STAGE && a.fuse_hazard == 2 && a.wpg && (blk % a.wpg) >= a.head && sink.ntau_out > 0) {
        // A tail wave (not a grid's head wave) normalises its columns' hazard rows itself once
        // every lane has solved — hazard_norm_kernel's operation, the same bits.  The tail waves
        // end long before the head waves that set the launch's length, so the pass (≈1 ms of
        // latency-bound loads per lane) is hidden; the head waves' columns are left to a small
        // hazard_norm_kernel launch after the learning (LearnArgs::part 1).  Eight entries per
        // round keep eight loads of each row in flight.
        double* __restrict__ H = L.hr + row;
        const double* __restrict__ HI = L.hrI + row;
        const int nt = sink.ntau_out;
        const double p = a.p, omp = 1.0 - p, ie = HI[nt - 1];
        for (int i0 = 0; i0 < nt; i0 += 8) {
            double h[8], q[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                h[k] = i0 + k < nt ? H[i0 + k] : 0.0;
                q[k] = i0 + k < nt ? HI[i0 + k] : 0.0;
            }
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (i0 + k < nt) H[i0 + k] = h[k] / ((p * q[k]) + (omp * ie));
        }
    }
    }
}

// Fused hazard, second half: HR_i = num_i / (p·I_i + (1 − p)·I_η) over every τ̄ entry the
// learning kernel streamed (num_i in the HR row, I_i in the hrI row; I_η = the last I).  Fully
// parallel and HBM-streaming (≈20 µs per 2048-column grid) — unlike hazard_kernel, whose
// workgroups hold CU slots for the length of a serial scan while equilibria are running.
constexpr int HN_BLOCK = 256, HN_UNROLL = 4;
__global__ __launch_bounds__(HN_BLOCK) void hazard_norm_kernel(LearnArgs a, LearnBufs L)
{
    // a.part == 1: only the columns of each grid's head waves (the rest normalised by their
    // learning waves, learn_logistic_kernel with fuse_hazard 2): block → grid's head column
    const int hc = 64 * a.head;
    const int b = a.part == 1 ? (int)(blockIdx.x / hc) * 64 * a.wpg + (int)(blockIdx.x % hc) : (int)blockIdx.x;
    const int nt = L.n_tau[b];
    if (nt <= 0) return;
    const size_t row = (size_t)b * (size_t)L.cap;
    double* __restrict__ H = L.hr + row;
    const double* __restrict__ HI = L.hrI + row;
    const double p = a.p, omp = 1.0 - p, ie = HI[nt - 1];
    for (int i0 = threadIdx.x; i0 < nt; i0 += HN_BLOCK * HN_UNROLL) {
        double h[HN_UNROLL], q[HN_UNROLL];
#pragma unroll
        for (int k = 0; k < HN_UNROLL; k++) {
            const int i = i0 + k * HN_BLOCK;
            h[k] = i < nt ? H[i] : 0.0;
            q[k] = i < nt ? HI[i] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < HN_UNROLL; k++) {
            const int i = i0 + k * HN_BLOCK;
            if (i < nt) H[i] = h[k] / ((p * q[k]) + (omp * ie));
        }
    }
}

// ============================================================================
// Hazard kernel — hazard_rate (solver.jl:153-185) for one β column per
// workgroup: τ̄ = knots ≤ η (+ η), pdf g = βG(1−G) (learning.jl:170), then
// e = exp(λτ̄)·g, the cumulative trapezoid (sequential, in the reference's
// order) and HR = (p·exp(λτ̄))·g / (p·I + (1−p)·I_η).
// ============================================================================
constexpr int kEqWide = 768; // lanes per equilibrium workgroup on wide u tiles
constexpr int kEqMinW = 6;    // waves per SIMD the baseline equilibrium kernel must fit (two 12-wave blocks per CU)
constexpr int HZ_BLOCK = 256;
constexpr int HZ_LDS = 1024; // τ̄ knots per LDS chunk of the hazard kernel
constexpr int HZ_REG = 16;   // τ̄ knots per thread held in registers (ntau <= 4096: one pass over HBM)
constexpr int EQ_TILE = 4096; // u values per equilibrium block (one block per β column up to this)
constexpr int kAwWin = 6;     // 8-blocks each side of the predicted AW peak evaluated first

// I_k = I_{k-1} + term_k over s_I[0, cn) in place, left to right (the reference's rounding
// order), by the 64 lanes of one wave: lane l holds terms [16l, 16l + 16) in registers and
// the running integral passes from lane to lane — in round r only lane r adds (16 dependent
// adds), then v_readlane broadcasts its I.  The chain is the adds plus one broadcast per 16
// terms; a one-lane scan out of LDS waits on an LDS round trip every few terms instead.
// Call with all 64 lanes of the wave active; I must be wave-uniform (and is on return).
constexpr int HZ_LANE = HZ_LDS / 64; // terms per lane (16)
__device__ __forceinline__ double hz_bcast(double x, int lane)
{
    const uint64_t u = sbr_dbits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), lane);
    return sbr_bitsd(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void hz_scan_wave(double* s_I, int cn, double& I)
{
    const int lane = threadIdx.x & 63, base = lane * HZ_LANE;
    double v[HZ_LANE];
#pragma unroll
    for (int j = 0; j < HZ_LANE; j++) v[j] = base + j < cn ? s_I[base + j] : 0.0;
    const int rounds = (cn + HZ_LANE - 1) / HZ_LANE;
    double acc = I;
    for (int r = 0; r < rounds; r++) {
        if (lane == r) {
            // the tail past cn adds +0.0, which leaves I (>= +0) unchanged
#pragma unroll
            for (int j = 0; j < HZ_LANE; j++) { acc = acc + v[j]; v[j] = acc; }
        }
        acc = hz_bcast(acc, r);
    }
    I = acc;
#pragma unroll
    for (int j = 0; j < HZ_LANE; j++)
        if (base + j < cn) s_I[base + j] = v[j];
}

#ifdef SBR_HZ_PROF // per-block phase cycles of the hazard kernel (tools/ubench_hazard.hip)
__device__ long long g_hzprof[8192 * 6];
#define HZ_T0 long long hz_tp = __builtin_amdgcn_s_memtime()
#define HZ_STAMP(ph)                                                                                  \
    do {                                                                                              \
        const long long hz_now = __builtin_amdgcn_s_memtime();                                        \
        if (threadIdx.x == 0) g_hzprof[(size_t)blockIdx.x * 6 + (ph)] += hz_now - hz_tp;              \
        hz_tp = hz_now;                                                                               \
    } while (0)
#else
#define HZ_T0
#define HZ_STAMP(ph)
#endif
// hazard_rate of column b by one workgroup of NT >= HZ_BLOCK threads (threads past HZ_BLOCK
// only take part in the barriers): the τ̄ grid in chunks of HZ_LDS knots, e_i·g_i and the
// trapezoid terms formed in parallel into LDS, one wave adds the terms left to right (the
// reference's rounding order), and a last parallel pass turns the partial integrals into
// HR_i.  LDS scratch: s_eg, s_t [HZ_LDS + 1], s_I [HZ_LDS], s_Ieta [1].  Every early
// return is uniform over the workgroup.
template <int NT, bool REGS = true>
__device__ __forceinline__ void hazard_column(const int b, const double BETA, const double ETA, const LearnArgs& a,
                                              const LearnBufs& L, double* s_eg, double* s_t, double* s_I,
                                              double* s_Ieta)
{
    static_assert(NT >= HZ_BLOCK, "hazard_column needs HZ_BLOCK threads");
    const int tid = threadIdx.x;
    const bool act = tid < HZ_BLOCK;
    HZ_T0;
    const int n = L.n_knots[b];
    const uint32_t st = L.status[b];
    if (st & SBR_ARG_INVALID) return; // learn kernel already wrote the row
    const size_t row = (size_t)b * (size_t)L.cap;
    const double* __restrict__ T = L.t + row;
    const double* __restrict__ Gv = L.G + row;
    double* __restrict__ H = L.hr + row;
    const double p = a.p, lam = a.lam;
    const int m = L.n_le[b]; // #knots ≤ η (searchsortedlast + 1), counted by the learning kernel
    bool oob = false, push;
    if (m < n) {
        push = (m == 0) || T[m - 1] != ETA; // solver.jl:159
        oob = (m == 0);                       // pdf(η) with η < t_0
    } else {
        push = (m == 0) || T[m - 1] != ETA;
        oob = push;                           // no knot beyond η to interpolate pdf(η)
    }
    const int ntau = m + (push ? 1 : 0);
    if (oob) {
        if (tid == 0) {
            L.status[b] = st | SBR_OOB;
            L.n_tau[b] = 0;
            L.n_le[b] = 0;
        }
        return;
    }
    // the pdf at knot i: compute_pdf_symbolic_baseline's βG(1 − G) (learning.jl:161-173), or the
    // caller's values (a.pdf: the interpolant of another pdf on the same knots)
    const double* __restrict__ PD = a.pdf ? a.pdf + row : nullptr; // the caller's pdf rows, laid out like G
    auto pdf_k = [&](int i) -> double {
        if (PD) return PD[i];
        const double x = Gv[i];
        return (BETA * x) * (1.0 - x);
    };
    auto pdf_at = [&](int i) -> double {
        if (i < m) return pdf_k(i);
        // η on bracket [m-1, m]
        const double g0 = pdf_k(m - 1);
        const double g1 = pdf_k(m);
        const double d = (ETA - T[m - 1]) / (T[m] - T[m - 1]);
        return g0 * (1.0 - d) + g1 * d;
    };
    auto tau_at = [&](int i) -> double { return i < m ? T[i] : ETA; };
    // Global reads are batched (unrolled loops, every load of a batch in flight before the
    // first use): the knots were written by another XCD's learning wave, so each one costs an
    // L2 miss, and one dependent miss per knot per thread would dominate the kernel.
    HZ_STAMP(0);
    if (REGS && ntau <= HZ_BLOCK * HZ_REG) {
        // Every τ̄ knot of the column in registers (thread tid owns knots tid + 256·j): one
        // batch of global loads, the chunks fed to LDS from registers, I_i read back into
        // registers, HR written once.
        double tv[HZ_REG], egv[HZ_REG], numv[HZ_REG], iv[HZ_REG], gk[HZ_REG];
        if (act) {
            // loads first, unconditionally (indices clamped into the knots ≤ η), so that all of
            // them are in flight at once; τ̄ = η and its interpolated pdf are selected after
            const double pdf_eta = m < n ? pdf_at(m) : 0.0; // m == n: η is a knot, not pushed
#pragma unroll
            for (int j = 0; j < HZ_REG; j++) {
                const int i = tid + HZ_BLOCK * j;
                const int ic = i < m ? i : m - 1;
                tv[j] = T[ic];
                gk[j] = PD ? PD[ic] : Gv[ic];
            }
#pragma unroll
            for (int j = 0; j < HZ_REG; j++) {
                const int i = tid + HZ_BLOCK * j;
                const double x = gk[j];
                const double ti = i < m ? tv[j] : ETA;
                const double g = i < m ? (PD ? x : (BETA * x) * (1.0 - x)) : pdf_eta;
                const double E = sbr_exp(lam * ti);
                tv[j] = ti;
                egv[j] = E * g;        // e_i = exp(λτ̄_i)·pdf_i
                numv[j] = (p * E) * g; // the HR numerator (p·exp(λτ̄_i))·pdf_i
                iv[j] = 0.0;
            }
        }
        double I = 0.0;
        constexpr int RPC = HZ_LDS / HZ_BLOCK; // register slots per LDS chunk
#pragma unroll
        for (int c = 0; c < HZ_REG / RPC; c++) {
            const int c0 = c * HZ_LDS;
            if (c0 < ntau) { // uniform
                const int cn = ntau - c0 < HZ_LDS ? ntau - c0 : HZ_LDS;
                if (act) {
#pragma unroll
                    for (int r = 0; r < RPC; r++) {
                        const int k = tid + HZ_BLOCK * r;
                        s_t[k + 1] = tv[c * RPC + r];
                        s_eg[k + 1] = egv[c * RPC + r];
                    }
                    if (c > 0 && tid == HZ_BLOCK - 1) { // knot c0 − 1 is this thread's last slot
                        s_t[0] = tv[c * RPC - 1];
                        s_eg[0] = egv[c * RPC - 1];
                    }
                }
                __syncthreads();
                HZ_STAMP(1);
                if (act)
                    for (int k = tid; k < cn; k += HZ_BLOCK)
                        s_I[k] = c0 + k == 0 ? 0.0 : (0.5 * (s_eg[k] + s_eg[k + 1])) * (s_t[k + 1] - s_t[k]);
                __syncthreads();
                HZ_STAMP(2);
                if (tid < 64) hz_scan_wave(s_I, cn, I);
                __syncthreads();
                HZ_STAMP(3);
                if (act) {
#pragma unroll
                    for (int r = 0; r < RPC; r++) {
                        const int k = tid + HZ_BLOCK * r;
                        if (k < cn) iv[c * RPC + r] = s_I[k];
                    }
                }
                __syncthreads(); // the chunk's LDS is reused
                HZ_STAMP(4);
            }
        }
        if (tid == 0) {
            s_Ieta[0] = I;
            L.n_tau[b] = ntau;
            L.n_le[b] = m;
        }
        __syncthreads();
        const double Ieta = s_Ieta[0], omp = 1.0 - p;
        if (act) {
#pragma unroll
            for (int j = 0; j < HZ_REG; j++) {
                const int i = tid + HZ_BLOCK * j;
                if (i < ntau) H[i] = numv[j] / ((p * iv[j]) + (omp * Ieta));
            }
        }
        HZ_STAMP(5);
        return;
    }
    double I = 0.0, egprev = 0.0, tprev = 0.0; // thread 0: running integral; the chunk's last e·g, τ̄
    for (int c0 = 0; c0 < ntau; c0 += HZ_LDS) {
        const int cn = ntau - c0 < HZ_LDS ? ntau - c0 : HZ_LDS;
        if (tid == 0) { s_eg[0] = egprev; s_t[0] = tprev; }
        if (act) {
#pragma unroll 4
            for (int k = tid; k < cn; k += HZ_BLOCK) {
                const int i = c0 + k;
                const double ti = tau_at(i);
                s_t[k + 1] = ti;
                s_eg[k + 1] = sbr_exp(lam * ti) * pdf_at(i); // e_i = exp(λτ̄_i)·pdf_i
            }
        }
        __syncthreads();
        HZ_STAMP(1);
        // trapezoid term of i pairs e_{i-1}, e_i (solver.jl:173-175); term_0 = 0
        if (act)
            for (int k = tid; k < cn; k += HZ_BLOCK)
                s_I[k] = c0 + k == 0 ? 0.0 : (0.5 * (s_eg[k] + s_eg[k + 1])) * (s_t[k + 1] - s_t[k]);
        __syncthreads();
        HZ_STAMP(2);
        if (tid < 64) hz_scan_wave(s_I, cn, I); // I_i = I_{i-1} + term_i, left to right
        if (tid == 0) {
            egprev = s_eg[cn];
            tprev = s_t[cn];
        }
        __syncthreads();
        HZ_STAMP(3);
        if (act)
            for (int k = tid; k < cn; k += HZ_BLOCK) H[c0 + k] = s_I[k]; // I_i parked in the HR row
        __syncthreads(); // the chunk's LDS is reused
        HZ_STAMP(4);
    }
    if (tid == 0) {
        s_Ieta[0] = I;
        L.n_tau[b] = ntau;
        L.n_le[b] = m;
    }
    __syncthreads();
    // HR_i = (p·exp(λτ̄_i))·pdf_i / (p·I_i + (1 − p)·I_η); each thread reads back the I_i it parked
    const double Ieta = s_Ieta[0], omp = 1.0 - p;
    if (act) {
#pragma unroll 4
        for (int i = tid; i < ntau; i += HZ_BLOCK) {
            const double E = sbr_exp(lam * tau_at(i));
            H[i] = ((p * E) * pdf_at(i)) / ((p * H[i]) + (omp * Ieta));
        }
    }
    HZ_STAMP(5);
}

__global__ __launch_bounds__(HZ_BLOCK) void hazard_kernel(const double* __restrict__ beta,
                                                          const double* __restrict__ eta, LearnArgs a, LearnBufs L)
{
    // 24 KiB of LDS per block, so hazard blocks of the next batch still fit beside two
    // equilibrium blocks on a CU
    __shared__ double s_eg[HZ_LDS + 1]; // s_eg[k + 1] = e·g of knot c0 + k; s_eg[0] that of knot c0 − 1
    __shared__ double s_t[HZ_LDS + 1];  // τ̄ likewise
    __shared__ double s_I[HZ_LDS];
    __shared__ double s_Ieta;
    __builtin_amdgcn_s_setprio(3);
    const int b = blockIdx.x;
    hazard_column<HZ_BLOCK>(b, beta[b], eta[b], a, L, s_eg, s_t, s_I, &s_Ieta);
}

// ============================================================================
// Equilibrium kernel
// ============================================================================
struct PointResult {
    double xi, tin, tout, aw, tol;
    uint32_t status;
    int iters;
};

// range check of an interpolation argument; returns false (and flags) when
// Interpolations' Throw() extrapolation would raise.
__device__ __forceinline__ bool in_range(double x, double tlo, double thi, bool trunc, uint32_t& flag)
{
    if (x >= tlo && x <= thi) return true;
    flag |= (trunc && x > thi) ? SBR_ENGINE_TRUNC : SBR_OOB;
    return false;
}

// Per-workgroup summaries staged in LDS next to the knot grid (null = unavailable):
//   hmax/hmin  per 64-entry block of HR(τ̄): max over non-NaN entries / min with NaN as −∞,
//              i.e. "some entry > u" ⇔ hmax > u and "every entry > u" ⇔ hmin > u;
//   pmc/smc    per 64-knot block of G: prefix max / suffix min over blocks (NaN-propagating).
struct Summ {
    const double* hmax;
    const double* hmin;
    const double* pmc;
    const double* smc;
    bool mono; // G nondecreasing over the knots (no NaN): prefix max / suffix min are knot values
    double t_half; // time where G crosses 1/2 (lerp inverse), NaN if it does not: AW peak predictor
    // aw_scan's preconditions: no NaN in G, 0 <= G[0], G[n−1] <= 2 (the 1e-14 rounding margin),
    // t[k+2] − t[k] > 1e-15·t[n−1] (a shifted τ̄ argument stays below the knot after next) and a
    // drawdown bound dd <= 1e-12 (Tsit5 at eps() leaves ulp-sized decreases in the saturated tail
    // of G on ≈20 % of the Fig 5 columns: G[k] <= G[k'] + dd for every k < k')
    bool scan;
    double dd;
    bool bnb; // the branch-and-bound bounds are available (mono, or the prefix/suffix tables built)
    // aw_scan's knot offset for AW_OUT(b_j) <= G[j + koff]: 1 when consecutive knots are more than
    // 1e-15·t[n−1] apart (b_j then lies below t[j + 1]: bracket <= j), else 2 (knots 2 apart)
    int koff;
    // prefix / suffix extremes of the HR block summaries: hpm = prefix max of hmax,
    // hpn = prefix min of hmin, hsm = suffix max of hmax, hsn = suffix min of hmin, over nbh
    // blocks; null: the linear block scans
    const double* hpm;
    const double* hpn;
    const double* hsm;
    const double* hsn;
    int nbh;
};

template <class P>
__device__ __forceinline__ void solve_from_buffers(P T, P G, P H, const Summ& S, const int n, const int ntau,
                                                   const int nle, const double ETA, const double T1, const bool trunc,
                                                   const double u, const double kappa, const int max_iters,
                                                   const uint32_t lbits, PointResult& r, double* __restrict__ aw_path,
                                                   const int diag, const double tin, const double tout);

// smallest k in [0, hi] with key(k) >= x, for a nondecreasing key with key(hi) >= x: gallop
// down from hi, then bisect
template <class F>
__device__ __forceinline__ int first_ge_down(F key, int hi, double x)
{
    int top = hi, lo = hi - 1, step = 1; // key(top) >= x; answer in (lo, top]
    while (lo >= 0 && key(lo) >= x) {
        top = lo;
        step <<= 1;
        lo = top - step;
    }
    if (lo < -1) lo = -1;
    while (top - lo > 1) {
        const int mid = (lo + top) >> 1;
        if (key(mid) >= x) top = mid;
        else lo = mid;
    }
    return top;
}

// AW_max (solver.jl:553-576) over τ̄ knots [0, ntau) by an outward scan from the predicted
// peak knot c, for a G with Summ::scan's preconditions (nondecreasing up to the drawdown dd:
// every bound below is widened by dd, and the margin is 1e-14 + 4·dd).  AW_cum(τ̄_i) =
// AW_OUT(b_i) − AW_IN(a_i) + G(0) with a_i = (τ̄_i − ξ) + icc ≤ b_i = (τ̄_i − ξ) + occ ≤ τ̄_i + ulp,
// both nondecreasing in i, so
//   right of the last evaluated knot i:  AW_OUT(b_j) ≤ G[j + 2] and AW_IN(a_j) ≥ AW_IN(a_i);
//   left of it:                         AW_OUT(b_j) ≤ AW_OUT(b_i) and AW_IN(a_j) ≥ G[bracket(a_j)].
// A knot is evaluated exactly (the same operations as eval_range) only where these bounds
// (+ the 1e-14 rounding margin) do not already put it at or below the running maximum; runs
// of knots the bounds dismiss are skipped with one search in G (right) or in G and τ̄ (left).
// The maximum equals the exhaustive one bit for bit (G has no NaN here).
// (A knot offset 0 for the AW_OUT bound inside [ξ/2, 2ξ], where b_i = t[i] exactly, halved the exact
// evaluations and was slower: an exact evaluation costs about what a bounded trip costs,
// profiles/experiments/r05_d_*)
template <class P>
__device__ __forceinline__ void aw_scan(P T, P G, const int n, const int ntau, const int nle, const double ETA,
                                        const double xi, const double icc, const double occ, const double G0,
                                        const double dd, const int c, double& mx, int& nev, const int koff = 2)
{
    const double M = 1e-14 + 4.0 * dd;
    auto tau = [&](int i) -> double { return i < nle ? T[i] : ETA; };
    auto av_of = [&](int i) -> double { return (tau(i) - xi) + icc; };
    // a(τ̄_i)'s bracket window: k = min(searchsortedlast(t, x), n − 2), its two knots (t, G)
    int ka;
    double ta0, ta1, ga0, ga1;
    auto seek = [&](int hint, double x) {
        ka = ssl_near(T, n, hint, x);
        ka = ka < n - 2 ? ka : n - 2;
        ta0 = T[ka]; ta1 = T[ka + 1]; ga0 = G[ka]; ga1 = G[ka + 1];
    };
    auto fwd = [&](double x) {
        while (ka < n - 2 && ta1 <= x) { ka++; ta0 = ta1; ga0 = ga1; ta1 = T[ka + 1]; ga1 = G[ka + 1]; }
    };
    auto bwd = [&](double x) {
        while (ka > 0 && ta0 > x) { ka--; ta1 = ta0; ga1 = ga0; ta0 = T[ka]; ga0 = G[ka]; }
    };
    // exact AW_cum(τ̄_i) with the a window at a_i's bracket; b's bracket is searched from i
    double awin = 0.0, awout = 0.0;
    auto exact = [&](int i, double av, double xa) -> double {
        const double ti = tau(i);
        const double bv = (ti - xi) + occ;
        const double xb = bv > 0 ? bv : 0.0;
        // b(τ̄_i) is τ̄_i = t[i] itself whenever τ̄_i − ξ is exact: bracket i, no search
        int kb = (i < nle && xb == ti) ? i : ssl_near(T, n, i, xb);
        kb = kb < n - 2 ? kb : n - 2;
        const double tb0 = T[kb], tb1 = T[kb + 1], gb0 = G[kb], gb1 = G[kb + 1];
        const double da = (xa - ta0) / (ta1 - ta0);
        const double gi = ga0 * (1.0 - da) + ga1 * da;
        double go;
        if (xb == tb0) go = gb0 * 1.0 + gb1 * 0.0;
        else { const double db = (xb - tb0) / (tb1 - tb0); go = gb0 * (1.0 - db) + gb1 * db; }
        awin = av >= 0 ? gi : 0.0;
        awout = bv >= 0 ? go : 0.0;
        nev++;
        return (awout - awin) + G0;
    };
    // knot c
    {
        const double av = av_of(c), xa = av > 0 ? av : 0.0;
        seek(c, xa);
        const double v = exact(c, av, xa);
        if (v > mx) mx = v;
    }
    const int kc = ka;
    const double ub_left = awout;
    // right of c
    double LA = awin; // lower bound of AW_IN(a_j) for every j >= i
    for (int i = c + 1; i < ntau;) {
        const double ti = tau(i);
        const double av = (ti - xi) + icc, xa = av > 0 ? av : 0.0;
        fwd(xa);
        const double lb = av >= 0 ? ga0 : 0.0;
        LA = LA > lb ? LA : lb;
        const double V = (((mx - G0) + LA) - M) - dd; // G[k] <= V: every knot up to k is <= V + dd
        const int k2 = i + koff < n - 1 ? i + koff : n - 1;
        if (G[k2] > V) {
            const double v = exact(i, av, xa);
            if (v > mx) mx = v;
            LA = awin;
            i++;
            continue;
        }
        // every knot j with G[min(j + 2, n − 1)] <= V is at or below mx: skip to the first other
        const int kl = ssl_gallop(G, n, k2, V);
        if (kl >= n - 1) break;
        // G[kl + 1] > V: the first knot whose bound is not dismissed
        const int inext = kl + 1 - koff;
        const double an = av_of(inext);
        seek(ka + (inext - i), an > 0 ? an : 0.0);
        i = inext;
    }
    // left of c
    double UB = ub_left; // upper bound of AW_OUT(b_j) for every j <= i
    {
        const double av = av_of(c);
        seek(kc, av > 0 ? av : 0.0);
    }
    for (int i = c - 1; i >= 0;) {
        const double ti = tau(i);
        const int k2 = i + koff < n - 1 ? i + koff : n - 1;
        const double g2 = G[k2] > 0.0 ? G[k2] : 0.0;
        UB = UB < g2 ? UB : g2;
        const double Vp = (((UB + G0) + M) - mx) + dd; // AW_IN(a_j) >= G[bracket(a_j)] − dd
        if (!(Vp - dd > 0.0)) break; // AW_IN(a_j) >= 0 for every j: all pruned
        const double av = (ti - xi) + icc, xa = av > 0 ? av : 0.0;
        bwd(xa);
        const double lb = av >= 0 ? ga0 : 0.0;
        if (!(lb >= Vp)) {
            const double v = exact(i, av, xa);
            if (v > mx) mx = v;
            UB = UB < awout ? UB : awout;
            i--;
            continue;
        }
        // knots j <= i with a_j >= t[k*] (k* = first knot with G >= Vp) are pruned
        const int ks = first_ge_down([&](int k) { return G[k]; }, ka, Vp);
        const double tk = T[ks];
        const int j = first_ge_down(av_of, i, tk);
        if (j == 0) break;
        const int inext = j - 1;
        const double an = av_of(inext);
        seek(ks, an > 0 ? an : 0.0);
        i = inext;
    }
}

// compute_ξ (solver.jl:308-376) from an arbitrary first iterate ξ_guess (the single-point kernel's
// knots-in calls only: the sweep kernel carries none of this): the reference's iteration as
// written, every lookup bracketed by a search over the whole grid (the oracle's compute_xi).  A
// lookup outside [t[0], t[n−1]] — G at a constrained time, searchsortedlast(grid, ξ_old) below the
// first knot or at the last, the ε probes — is the interpolant's BoundsError.
template <class P>
__device__ __forceinline__ void bisect_plain(P T, P G, const int n, const double tlo, const double thi,
                                             const bool trunc, const double tin, const double tout,
                                             const double guess, const double kappa, const double tolerance,
                                             const int max_iters, PointResult& r, uint32_t& flag, uint32_t& s,
                                             double& xi, double& tolr)
{
    double xnew = guess, xmin = tin, xmax = tout;
    for (int iter = 1; iter <= max_iters; iter++) {
        r.iters = iter;
        if (collapsed(xmin - xmax)) { s = SBR_NO_RUN_COLLAPSE; return; }
        if (iter == max_iters - 1) { s = SBR_NO_RUN_MAXITER; return; }
        const double xo = xnew;
        const double ic = dmin(tin, xo), oc = dmin(tout, xo);
        double Goc = 0.0, Gic = 0.0;
        if (in_range(oc, tlo, thi, trunc, flag)) Goc = lerp_at(T, G, n, ssl_range(T, 0, n - 1, oc), oc);
        if (in_range(ic, tlo, thi, trunc, flag)) Gic = lerp_at(T, G, n, ssl_range(T, 0, n - 1, ic), ic);
        if (!(xo >= tlo)) { flag |= SBR_OOB; return; } // searchsortedlast = 0: grid[0]
        const int j = ssl_range(T, 0, n - 1, xo);
        if (j + 1 >= n) { flag |= trunc ? SBR_ENGINE_TRUNC : SBR_OOB; return; }
        const double eps = T[j + 1] - T[j];
        const double xoe = oc + eps, xie = ic + eps;
        const bool oke = in_range(xoe, tlo, thi, trunc, flag);
        const bool oki = in_range(xie, tlo, thi, trunc, flag);
        if (flag) return;
        const double AW = Goc - Gic;
        const double err = AW - kappa;
        if (fabs(err) <= tolerance) {
            double Goce = 0.0, Gice = 0.0;
            if (oke) Goce = lerp_at(T, G, n, ssl_range(T, 0, n - 1, xoe), xoe);
            if (oki) Gice = lerp_at(T, G, n, ssl_range(T, 0, n - 1, xie), xie);
            if (Goce - Gice >= AW) { s = SBR_RUN; xi = xo; tolr = fabs(err); }
            else s = SBR_FALSE_EQ;
            return;
        } else if (err > 0) {
            xmax = xo; xnew = 0.5 * (xo + xmin);
        } else {
            xmin = xo; xnew = 0.5 * (xo + xmax);
        }
    }
}

template <class P>
__device__ __forceinline__ void solve_point(P T, P G, P H, const Summ& S, const int n, const int ntau,
                                            const int nle, const double ETA, const double T1, const bool trunc,
                                            const double u, const double kappa, const int max_iters,
                                            const uint32_t lbits, PointResult& r, double* __restrict__ aw_path,
                                            const int diag)
{
    r.xi = NAN; r.aw = NAN; r.tol = INFINITY; r.iters = 0; r.status = 0;
    (void)0;

    // ---------------- optimal_buffer: crossings of HR(τ̄) with u ----------------
    bool any, all;
    int fa, la, cin, cout;
    if (S.hpm) {
        buffer_scan_bs(H, S, S.hpm, S.hpn, S.hsm, S.hsn, S.nbh, ntau, u, any, all, fa, la, cin, cout);
    } else if (S.hmax) {
        buffer_scan_blocked(H, S, ntau, u, any, all, fa, la, cin, cout);
    } else {
        any = false; all = true;
        bool prev = false;
        fa = la = cin = cout = -1;
        for (int i = 0; i < ntau; i++) {
            const bool ab = H[i] > u;
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
    auto tau = [&](int i) -> double { return i < nle ? T[i] : ETA; };
    double tin, tout;
    if (!any) {
        tin = T1; tout = T1;
    } else if (all) {
        tin = tau(0); tout = tau(ntau - 1);
    } else {
        tin = T1; tout = T1;
        if (cin >= 0) {
            const double t0 = tau(cin), t1 = tau(cin + 1), h0 = H[cin], h1 = H[cin + 1];
            tin = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
        }
        if (cout >= 0) {
            const double t0 = tau(cout), t1 = tau(cout + 1), h0 = H[cout], h1 = H[cout + 1];
            tout = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
        }
        if (tin == T1) tin = tau(fa);
        if (tout == T1) tout = tau(la);
    }
    r.tin = tin;
    r.tout = tout;
    if (diag & 1) return;
    solve_from_buffers(T, G, H, S, n, ntau, nle, ETA, T1, trunc, u, kappa, max_iters, lbits, r, aw_path, diag,
                       tin, tout);
}

// solve_equilibrium_baseline from the buffer times on (solver.jl:429-462) + get_AW / AW_max:
// no run if τ̄_IN == τ̄_OUT, else compute_ξ on G and AW_max on the τ̄ grid.
template <class P>
__device__ __forceinline__ void solve_from_buffers(P T, P G, P H, const Summ& S, const int n, const int ntau,
                                                   const int nle, const double ETA, const double T1, const bool trunc,
                                                   const double u, const double kappa, const int max_iters,
                                                   const uint32_t lbits, PointResult& r, double* __restrict__ aw_path,
                                                   const int diag, const double tin, const double tout)
{
    const double tlo = T[0], thi = T[n - 1];
    auto tau = [&](int i) -> double { return i < nle ? T[i] : ETA; };
    if (tin == tout) {
        r.status = SBR_NO_RUN_HR_BELOW_U | SBR_CONVERGED | lbits;
        r.tol = 0.0;
        return;
    }

    // ---------------- compute_ξ: bisection with bracketed lookups ----------------
    uint32_t flag = 0;
    const double tolerance = 10.0 * sbr_jl_eps(kappa);
    double xnew = (tin + tout) / 2.0, xmin = tin, xmax = tout;
    const bool okmin = in_range(xmin, tlo, thi, trunc, flag);
    const bool okmax = in_range(xmax, tlo, thi, trunc, flag);
    if (!okmin || !okmax) {
        r.status = flag | lbits;
        return;
    }
    int jlo = ssl_range(T, 0, n - 1, xmin);
    int jhi = ssl_range(T, 0, n - 1, xmax);
    const int jtin = jlo;
    double c_ic_x = NAN, c_ic_v = 0.0;
    uint32_t s = SBR_NO_RUN_MAXITER;
    double xi = NAN, tolr = INFINITY;
    // Single-interval bisection.  Once the bracket is one knot interval [t0, t1) (jlo == jhi),
    // G(ξ) there is the line g0·(1 − δ) + g1·δ, and the error AW − κ of a midpoint is
    // e0 + s·(x − t0) up to a few ulps of the operands.  Every midpoint whose estimate is
    // farther than `lim` from zero has the sign of its estimate and is no terminal iterate
    // (|AW − κ| > tol): it moves xmin or xmax without the search, the lerp and its division.
    // Only the last few midpoints (|err| ≲ 1e-13) run the exact iteration below.  The
    // exact iteration's other effects are constant over the interval (ic = tin, oc = ξ,
    // ε = t1 − t0, the BoundsError tests of ξ + ε and tin + ε pass), checked on entry.
    // ea = s·x + c (c = e0 − s·t0, |s·t0| ≤ 16: the rounding of c and of the fma stays ≈1e-14, far
    // inside lim); f_s = NaN until the interval is reached: every comparison fails and the exact
    // iteration runs.  Lanes of a wave move through the same trips, the decided ones skipping
    // the exact body.
    double f_s = NAN, f_c = 0.0;
    const double f_lim = tolerance + 1e-13;
    for (int iter = 1; iter <= max_iters; iter++) {
        r.iters = iter;
        const double dd = xmin - xmax;
        if (collapsed(dd)) { s = SBR_NO_RUN_COLLAPSE; break; }
        if (iter == max_iters - 1) { s = SBR_NO_RUN_MAXITER; break; }
        const double xo = xnew;
        {
            const double ea = fma(f_s, xo, f_c);
            if (ea < -f_lim) { xmin = xo; xnew = 0.5 * (xo + xmax); continue; }
            if (ea > f_lim) { xmax = xo; xnew = 0.5 * (xo + xmin); continue; }
        }
        const double ic = dmin(tin, xo), oc = dmin(tout, xo);
        const int j = ssl_range(T, jlo, jhi, xo); // t[jlo] <= ξmin <= xo <= ξmax < t[jhi+1]
        // G(oc)
        bool ok = in_range(oc, tlo, thi, trunc, flag);
        int joc = (oc == xo) ? j : (ok ? ssl_range(T, 0, n - 1, oc) : 0);
        const double Goc = ok ? lerp_at(T, G, n, joc, oc) : 0.0;
        // G(ic) — ic == tin for every iterate of a valid bracket; cached by value
        double Gic = 0.0;
        int jic = 0;
        if (in_range(ic, tlo, thi, trunc, flag)) {
            jic = (ic == tin) ? jtin : (ic == xo ? j : ssl_range(T, 0, n - 1, ic));
            if (ic == c_ic_x) Gic = c_ic_v;
            else { Gic = lerp_at(T, G, n, jic, ic); c_ic_x = ic; c_ic_v = Gic; }
        }
        // ε = local knot spacing at ξ_old (solver.jl:336-338)
        if (j + 1 >= n) { flag |= trunc ? SBR_ENGINE_TRUNC : SBR_OOB; break; }
        const double eps = T[j + 1] - T[j];
        const double xoe = oc + eps, xie = ic + eps;
        // the slope probe AW(ξ + ε) only decides the terminal iterate (solver.jl:345-352);
        // its lookups' BoundsError checks still run every iterate, in the reference's order
        const bool oke = in_range(xoe, tlo, thi, trunc, flag);
        const bool oki = in_range(xie, tlo, thi, trunc, flag);
        if (flag) break;
        const double AW = Goc - Gic;
        const double err = AW - kappa;
        if (fabs(err) <= tolerance) {
            double Goce = 0.0, Gice = 0.0;
            if (oke) Goce = lerp_at(T, G, n, ssl_gallop(T, n, joc, xoe), xoe);
            if (oki) Gice = lerp_at(T, G, n, ssl_gallop(T, n, jic, xie), xie);
            const double AWe = Goce - Gice;
            if (AWe >= AW) { s = SBR_RUN; xi = xo; tolr = fabs(err); }
            else s = SBR_FALSE_EQ;
            break;
        } else if (err > 0) {
            xmax = xo; jhi = j; xnew = 0.5 * (xo + xmin);
        } else {
            xmin = xo; jlo = j; xnew = 0.5 * (xo + xmax);
        }
        if (f_s != f_s && jlo == jhi && ic == tin && tin <= xmin && xmax <= tout && xmax + eps <= thi) {
            // j + 1 < n and ξ + ε, tin + ε in range were tested by this iteration
            const double t0 = T[j], g0 = G[j], g1 = G[j + 1];
            const double mag = dmax(dmax(fabs(g0), fabs(g1)), dmax(fabs(Gic), fabs(kappa)));
            if (mag <= 4.0 && eps > 0.0) { // finite, moderate operands (NaN fails): rounding ≤ 1e-14
                const double sl = (g1 - g0) / eps, st = sl * t0;
                if (fabs(st) <= 16.0) { // |c| ≤ 28: its rounding stays ≈1e-14
                    f_s = sl;
                    f_c = ((g0 - Gic) - kappa) - st;
                }
            }
        }
    }
    if (flag) { r.status = flag | lbits; return; }
    if (s != SBR_RUN) { r.status = s | lbits; return; }
    if (diag & 2) return;
    int nblk_eval = 0;

    // ---------------- get_AW on the HR grid + AW_max ----------------
    const double icc = (tin >= xi) ? xi : tin;
    const double occ = (tout > xi) ? xi : tout;
    if (!in_range(0.0, tlo, thi, trunc, flag)) { r.status = flag | lbits; return; }
    const double G0 = lerp_at(T, G, n, ssl_range(T, 0, n - 1, 0.0), 0.0);
    double mx = -INFINITY;
    auto xa_of = [&](int i) { const double v = (tau(i) - xi) + icc; return v > 0 ? v : 0.0; };
    auto xb_of = [&](int i) { const double v = (tau(i) - xi) + occ; return v > 0 ? v : 0.0; };
    // Brackets of a(τ̄_i) and b(τ̄_i) are searched from the last one found, moved by
    // the τ̄ distance (both are τ̄_i shifted by a constant, so they advance with i).
    int ra_i = 0, ra_j = 0, rb_i = 0, rb_j = 0;
    auto brk_a = [&](int i) { ra_j = ssl_near(T, n, ra_j + (i - ra_i), xa_of(i)); ra_i = i; return ra_j; };
    auto brk_b = [&](int i) { rb_j = ssl_near(T, n, rb_j + (i - rb_i), xb_of(i)); rb_i = i; return rb_j; };
    // exact AW_cum(τ̄_i) for i in [i0, i1), folded into the NaN-propagating max
    auto eval_range = [&](int i0, int i1) {
        // The brackets of a(τ̄_i) and b(τ̄_i) only move forward with i: keep each bracket's
        // two knots (t, G) in registers and slide them, so a knot costs the LDS loads of
        // the knots the brackets pass (≈1 per argument) instead of a fresh search + 4 lerp
        // operands each.  Bracket k = min(searchsortedlast, n − 2), as lerp_at clamps it.
        int ka = brk_a(i0), kb = brk_b(i0);
        ka = ka < n - 2 ? ka : n - 2;
        kb = kb < n - 2 ? kb : n - 2;
        double ta0 = T[ka], ta1 = T[ka + 1], ga0 = G[ka], ga1 = G[ka + 1];
        double tb0 = T[kb], tb1 = T[kb + 1], gb0 = G[kb], gb1 = G[kb + 1];
        for (int i = i0; i < i1; i++) {
            const double ti = tau(i);
            const double av = (ti - xi) + icc;
            const double bv = (ti - xi) + occ;
            const double xa = av > 0 ? av : 0.0;
            const double xb = bv > 0 ? bv : 0.0;
            if (!(xa <= thi) || !(xb <= thi)) { flag |= trunc ? SBR_ENGINE_TRUNC : SBR_OOB; return; }
            while (ka < n - 2 && ta1 <= xa) { ka++; ta0 = ta1; ga0 = ga1; ta1 = T[ka + 1]; ga1 = G[ka + 1]; }
            while (kb < n - 2 && tb1 <= xb) { kb++; tb0 = tb1; gb0 = gb1; tb1 = T[kb + 1]; gb1 = G[kb + 1]; }
            const double da = (xa - ta0) / (ta1 - ta0);
            const double gi = ga0 * (1.0 - da) + ga1 * da;
            // b(τ̄_i) = (τ̄_i − ξ) + ξ is τ̄_i itself whenever τ̄_i − ξ is exact (Sterbenz):
            // then δ = 0 and the lerp is G[j]·(1 − 0) + G[j+1]·0, no division
            double go;
            if (xb == tb0) go = gb0 * 1.0 + gb1 * 0.0;
            else { const double db = (xb - tb0) / (tb1 - tb0); go = gb0 * (1.0 - db) + gb1 * db; }
            const double awin = av >= 0 ? gi : 0.0;
            const double awout = bv >= 0 ? go : 0.0;
            const double v = (awout - awin) + G0;
            if (diag & 4) nblk_eval++;
            if (aw_path) aw_path[i] = v;
            if (mx == mx && (v != v || v > mx)) mx = v;
        }
        ra_j = ka; ra_i = i1 - 1;
        rb_j = kb; rb_i = i1 - 1;
    };
    // AW peak predictor (a logistic-shaped CDF): the continuous maximiser of
    // G(τ − s_out) − G(τ − s_in) sits where G(τ − s_out) + G(τ − s_in) = 1, i.e. at
    // τ* = t_half + (s_in + s_out)/2
    const double tstar = S.t_half + 0.5 * ((xi - icc) + (xi - occ));
    const bool predicted = tstar == tstar && tstar >= tau(0) && tstar <= tau(ntau - 1);
    const bool scan = S.scan && predicted;
    if (!S.pmc || aw_path || !(scan || S.bnb)) {
        eval_range(0, ntau); // exhaustive (single-point path mode, or summaries unavailable)
    } else {
        // Branch and bound over a 256/64/8 hierarchy of τ̄ ranges — the same maximum,
        // far fewer evaluations.  Every argument sequence is nondecreasing in i, so the
        // range check of the last τ̄ covers the whole path.
        const double al = (tau(ntau - 1) - xi) + icc, bl = (tau(ntau - 1) - xi) + occ;
        if (!((al > 0 ? al : 0.0) <= thi) || !((bl > 0 ? bl : 0.0) <= thi)) {
            flag |= trunc ? SBR_ENGINE_TRUNC : SBR_OOB;
        } else {
            // Upper bound of AW_cum over τ̄ indices [i0, i1]: AW_OUT ≤ max G over knots
            // ≤ bracket(b(τ̄_i1)) + 1, AW_IN ≥ min G over knots ≥ bracket(a(τ̄_i0)) (8-knot
            // prefix-max / suffix-min tables), plus a rounding margin far above the
            // ≈2e-15 the exact path can add.
            // When G is nondecreasing (every learning CDF of the configs) the prefix max up to
            // knot k is G[k] and the suffix min from k is G[k]: knot-exact bounds, loose by one
            // knot interval instead of an 8-knot block on each side.
            auto ub_rng = [&](int i0, int i1) -> double {
                const int ja = brk_a(i0), jb = brk_b(i1);
                const int kh = jb + 1 < n - 1 ? jb + 1 : n - 1, kl = ja < n - 2 ? ja : n - 2;
                const double hi = S.mono ? G[kh] : S.pmc[kh >> 3];
                const double lo = S.mono ? G[kl] : S.smc[kl >> 3];
                const double ub_out = hi > 0.0 ? hi : 0.0;
                const double lb_in = ((tau(i0) - xi) + icc) >= 0 ? lo : (lo < 0.0 ? lo : 0.0);
                return ((ub_out - lb_in) + G0) + 1e-14;
            };
            auto end_of = [&](int i0, int w) { return i0 + w < ntau ? i0 + w : ntau; };
            // pass 1: a first running maximum.  For a logistic-shaped CDF the continuous
            // maximiser of G(τ − s_out) − G(τ − s_in) sits where G(τ − s_out) + G(τ − s_in) = 1,
            // i.e. at τ* = t_half + (s_in + s_out)/2: evaluate the 8-blocks around it
            // (a heuristic — exactness comes from pass 2's bounds).  Otherwise descend the
            // bound hierarchy to the most promising 8-block.
            const int ic = predicted ? ssl_range(T, 0, (nle > 0 ? nle : 1) - 1, tstar < T[0] ? T[0] : tstar) : 0;
            if (scan) {
                aw_scan(T, G, n, ntau, nle, ETA, xi, icc, occ, G0, S.dd, ic < ntau ? ic : ntau - 1, mx, nblk_eval,
                        S.koff);
            } else
            {
            int b8 = -1, w0 = 0, w1 = 0;
            if (predicted) {
                const int c8 = (ic < ntau ? ic : ntau - 1) & ~7;
                w0 = c8 - 8 * kAwWin > 0 ? c8 - 8 * kAwWin : 0;
                w1 = end_of(c8, 8 * (kAwWin + 1));
                eval_range(w0, w1);
            } else {
                int bs = 0;
                double bu = -INFINITY;
                for (int i0 = 0; i0 < ntau; i0 += 256) {
                    const double ub = ub_rng(i0, end_of(i0, 256) - 1);
                    if (!(ub <= bu)) { bu = ub; bs = i0; }
                }
                int bb = bs;
                bu = -INFINITY;
                for (int i0 = bs; i0 < end_of(bs, 256); i0 += 64) {
                    const double ub = ub_rng(i0, end_of(i0, 64) - 1);
                    if (!(ub <= bu)) { bu = ub; bb = i0; }
                }
                b8 = bb;
                bu = -INFINITY;
                for (int i0 = bb; i0 < end_of(bb, 64); i0 += 8) {
                    const double ub = ub_rng(i0, end_of(i0, 8) - 1);
                    if (!(ub <= bu)) { bu = ub; b8 = i0; }
                }
                eval_range(b8, end_of(b8, 8));
            }
            // pass 2: every range whose bound beats the running max is refined
            for (int s0 = 0; s0 < ntau && !flag && mx == mx; s0 += 256) {
                const int se = end_of(s0, 256);
                if (ub_rng(s0, se - 1) <= mx) continue;
                for (int k0 = s0; k0 < se && !flag && mx == mx; k0 += 64) {
                    const int ke = end_of(k0, 64);
                    if (ub_rng(k0, ke - 1) <= mx) continue;
                    for (int i0 = k0; i0 < ke && !flag && mx == mx; i0 += 8) {
                        const int ie = end_of(i0, 8);
                        if (i0 == b8 || (i0 >= w0 && ie <= w1) || ub_rng(i0, ie - 1) <= mx) continue;
                        eval_range(i0, ie);
                    }
                }
            }
            }
        }
    }
    if (flag) { r.status = flag | lbits; return; }
    r.xi = xi;
    r.tol = tolr;
    r.aw = mx;
    r.status = SBR_RUN | SBR_CONVERGED | lbits;
    if (diag & 4) r.iters = nblk_eval;
}

// ============================================================================
// Interest-rate extension (src/extensions/interest_rates/)
// ============================================================================
// τ̄ grid view: knots ≤ η, then η (hazard_rate's grid, solver.jl:155-161)
template <class P>
struct TauView {
    P T;
    int nle;
    double eta;
    __device__ __forceinline__ double operator[](int i) const { return i < nle ? T[i] : eta; }
};

// Tsit5 dense-output coefficients (OrdinaryDiffEqTsit5 Tsit5Interp) — as oracle tsit5_dense
constexpr double R11 = 1.0, R12 = -2.763706197274826, R13 = 2.9132554618219126, R14 = -1.0530884977290216;
constexpr double R22 = 0.13169999999999998, R23 = -0.2234, R24 = 0.1017;
constexpr double R32 = 3.9302962368947516, R33 = -5.941033872131505, R34 = 2.490627285651253;
constexpr double R42 = -12.411077166933676, R43 = 30.33818863028232, R44 = -16.548102889244902;
constexpr double R52 = 37.50931341651104, R53 = -88.1789048947664, R54 = 47.37952196281928;
constexpr double R62 = -27.896526289197286, R63 = 65.09189467479366, R64 = -34.87065786149660;
constexpr double R72 = 1.5, R73 = -4.0, R74 = 2.5;

// the step's interpolant at Θ (saveat): Horner b_i(Θ), nested muladd sum
__device__ __forceinline__ double tsit5_dense(double th, double dt, double y0, double k1, double k2, double k3,
                                              double k4, double k5, double k6, double k7)
{
    const double th2 = th * th;
    const double b1 = th * fma(th, fma(th, fma(th, R14, R13), R12), R11);
    const double b2 = th2 * fma(th, fma(th, R24, R23), R22);
    const double b3 = th2 * fma(th, fma(th, R34, R33), R32);
    const double b4 = th2 * fma(th, fma(th, R44, R43), R42);
    const double b5 = th2 * fma(th, fma(th, R54, R53), R52);
    const double b6 = th2 * fma(th, fma(th, R64, R63), R62);
    const double b7 = th2 * fma(th, fma(th, R74, R73), R72);
    const double sum = fma(k1, b1, fma(k2, b2, fma(k3, b3, fma(k4, b4, fma(k5, b5, fma(k6, b6, k7 * b7))))));
    return fma(dt, sum, y0);
}

// hjb_equation! (value_function_solver.jl:86-95): dV = (h + δ)(1 − V) + max(u + rV − h, 0)
// with h = HR(τ̄) (gridded linear, Throw()); brackets galloped from the step's own.
template <class P>
struct ValueRhs {
    TauView<P> tau;
    P H;
    int ntau;
    double delta, r, u, tlo, thi;
    int jb;
    bool oob;
    __device__ __forceinline__ double hr(double t)
    {
        if (ntau < 2 || !(t >= tlo && t <= thi)) { oob = true; return (double)NAN; }
        const int j = (tau[jb] <= t) ? ssl_gallop(tau, ntau, jb, t) : ssl_range(tau, 0, jb, t);
        return lerp_at(tau, H, ntau, j, t);
    }
    __device__ __forceinline__ double eval(double t, double V)
    {
        const double h = hr(t);
        const double x = (u + r * V) - h;
        const double re = (x != x) ? x : (x > 0.0 ? x : 0.0); // Julia max(x, 0.0)
        return (h + delta) * (1.0 - V) + re;
    }
    __device__ __forceinline__ void prepare(double, double) {}
    __device__ __forceinline__ double stage(int, double ts, double V) { return eval(ts, V); }
    // ForwardDiff (oracle jac_value): max(x, 0.0) on a Dual keeps x iff 0 < x (or NaN);
    // J = −(h + δ) + (r | 0), ∂f/∂τ̄ = h'·(1 − V) + (−h' | 0), h' the HR interpolant's slope
    __device__ __forceinline__ void jac(double t, double V, double& J, double& dT)
    {
        double h = (double)NAN, hp = (double)NAN;
        if (ntau < 2 || !(t >= tlo && t <= thi)) {
            oob = true;
        } else {
            int j = (tau[jb] <= t) ? ssl_gallop(tau, ntau, jb, t) : ssl_range(tau, 0, jb, t);
            j = j > ntau - 2 ? ntau - 2 : (j < 0 ? 0 : j);
            const double t0 = tau[j], t1 = tau[j + 1], h0 = H[j], h1 = H[j + 1];
            const double d = (t - t0) / (t1 - t0);
            h = h0 * (1.0 - d) + h1 * d;
            const double rr = 1.0 / (t1 - t0);
            hp = h0 * (-rr) + h1 * rr;
        }
        const double x = (u + r * V) - h;
        const bool keep = (x != x) || (x > 0.0);
        J = (h + delta) * (-1.0) + (keep ? r : 0.0);
        dT = hp * (1.0 - V) + (keep ? -hp : 0.0);
    }
    __device__ __forceinline__ void accepted(double t)
    {
        if (ntau >= 2 && t >= tlo && t <= thi) jb = ssl_gallop(tau, ntau, jb, t);
    }
    static constexpr bool kFsalExact = false;
    static constexpr int kPinTableau = 0;
};

// The value function saved on the HR grid (saveat) streamed into optimal_buffer
// on h − rV (interest_rate_solver.jl:84-93, solver.jl:211-264): V(τ̄_i) and HR(τ̄_i)
// are their interpolants at their own knots (v_i·(1−0) + v_{i+1}·0, the last knot
// v_{n−2}·0 + v_{n−1}·1), so knot i is scanned once V_{i+1} is known.
template <class P>
struct SaveScan {
    TauView<P> tau;
    P H;
    int ntau;
    double r, u;
    double* vpath;   // single-point mode: every saved V (may be null)
    int next;        // grid index of the next saved value
    double vprev;    // V at knot next − 1 (its h − rV waits for V_next)
    double vprev2;   // V at knot next − 2
    int nh;          // h − rV values scanned
    double hprev;    // h − rV at knot nh − 1
    bool any, all;
    int fa, la, cin, cout;
    double tin_x, tout_x; // crossing lerps (valid when cin / cout ≥ 0)
    __device__ __forceinline__ void init(double V0)
    {
        next = 1; vprev = V0; vprev2 = 0.0; nh = 0; hprev = 0.0;
        if (vpath) vpath[0] = V0;
        any = false; all = true; fa = la = cin = cout = -1; tin_x = tout_x = 0.0;
    }
    __device__ __forceinline__ void scan(double hv)
    {
        const int i = nh;
        const bool ab = hv > u;
        any |= ab;
        all &= ab;
        if (ab) { if (fa < 0) fa = i; la = i; }
        if (i > 0) {
            const bool pab = hprev > u;
            const double t0 = tau[i - 1], t1 = tau[i];
            if (!pab && ab && cin < 0) { cin = i - 1; tin_x = t0 + ((u - hprev) * (t1 - t0)) / (hv - hprev); }
            if (pab && !ab) { cout = i - 1; tout_x = t0 + ((u - hprev) * (t1 - t0)) / (hv - hprev); }
        }
        hprev = hv;
        nh = i + 1;
    }
    // V_k saved (k = next): knot k − 1 is interior to V's grid now
    __device__ __forceinline__ void save(double v)
    {
        const int i = next - 1;
        if (vpath) vpath[next] = v;
        const double ti = tau[i], t1 = tau[i + 1];
        const double d = (ti - ti) / (t1 - ti);
        const double Vi = vprev * (1.0 - d) + v * d;
        scan(lerp_at(tau, H, ntau, i, ti) - r * Vi);
        vprev2 = vprev;
        vprev = v;
        next++;
    }
    // after the solve: the last saved knot (j = n − 2, δ = 1)
    __device__ __forceinline__ void finish()
    {
        const int i = next - 1;
        const double t0 = tau[i - 1], ti = tau[i];
        const double d = (ti - t0) / (ti - t0);
        const double Vi = vprev2 * (1.0 - d) + vprev * d;
        scan(lerp_at(tau, H, ntau, i, ti) - r * Vi);
    }
};

// solve_equilibrium_interest (interest_rate_solver.jl:51-150) for one u with r > 0:
// V on the HR grid, optimal_buffer on h − rV, then the baseline's compute_ξ / AW.
template <class P>
__device__ __forceinline__ void solve_interest_point(P T, P G, P H, const Summ& S, const int n, const int ntau,
                                                     const int nle, const double ETA, const double T1,
                                                     const bool trunc, const double u, const double kappa,
                                                     const int max_iters, const uint32_t lbits,
                                                     const InterestArgs& ia, PointResult& r, int64_t& nsteps,
                                                     double* __restrict__ aw_path, const int diag)
{
    r.xi = NAN; r.aw = NAN; r.tol = INFINITY; r.iters = 0; r.status = 0;
    nsteps = 0;
    const TauView<P> tau{T, nle, ETA};
    ValueRhs<P> f{tau, H, ntau, ia.delta, ia.r, u, ntau > 0 ? tau[0] : 0.0, ntau > 0 ? tau[ntau - 1] : 0.0, 0, false};
    const double V0 = (u + ia.delta) / (ia.r + ia.delta);
    SaveScan<P> sv{tau, H, ntau, ia.r, u, ia.v_path};
    sv.init(V0);
    // savevalues! with saveat = the HR grid: each pending grid point ≤ the new t is the
    // step's dense output at Θ = (s − tprev)/dt (Tsit5's or Rosenbrock23's), or u itself at t
    struct Saver {
        SaveScan<P>& sv;
        const TauView<P>& tau;
        int ntau;
        __device__ __forceinline__ bool start(double, double) { return true; }
        __device__ __forceinline__ bool step(bool acc, double tprev, double tn, double dt, double y0, double y1,
                                             const StepK& K, bool)
        {
            while (acc && sv.next < ntau && tau[sv.next] <= tn) {
                const double ts = tau[sv.next];
                const double th = (ts - tprev) / dt;
                sv.save(ts != tn ? (K.stiff ? ros23_dense(th, dt, y0, K.k[0], K.k[1])
                                            : tsit5_dense(th, dt, y0, K.k[0], K.k[1], K.k[2], K.k[3], K.k[4],
                                                          K.k[5], K.k[6]))
                                 : y1);
            }
            return true;
        }
    } saver{sv, tau, ntau};
    OdeOut vo;
    ode_scalar(f, saver, ntau > 0 ? tau[ntau - 1] : 0.0, V0, ia.rtol, ia.atol, ia.maxiters, vo);
    uint32_t vbits = vo.status;
    nsteps = vo.naccept + vo.nreject;
    if (ia.v_count) *ia.v_count = sv.next;
    if (f.oob) vbits |= SBR_OOB;
    const uint32_t bits = lbits | (vbits & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED));
    if ((vbits & SBR_OOB) || sv.next < 2) { // HR lookup past the grid / a 1-knot V interpolant: BoundsError
        r.status = SBR_OOB | bits;
        r.tin = NAN; r.tout = NAN;
        return;
    }
    sv.finish();
    const int ns = sv.nh;
    double tin, tout;
    if (!sv.any) {
        tin = T1; tout = T1;
    } else if (sv.all) {
        tin = tau[0]; tout = tau[ns - 1];
    } else {
        tin = sv.cin >= 0 ? sv.tin_x : T1;
        tout = sv.cout >= 0 ? sv.tout_x : T1;
        if (tin == T1) tin = tau[sv.fa];
        if (tout == T1) tout = tau[sv.la];
    }
    r.tin = tin;
    r.tout = tout;
    if (diag & 1) { r.status = bits; return; }
    solve_from_buffers(T, G, H, S, n, ntau, nle, ETA, T1, trunc, u, kappa, max_iters, bits, r, aw_path, diag, tin,
                       tout);
}

// The equilibria of u values [j0, j1) of column b by one workgroup of BLOCK threads (smem:
// the dynamic LDS slab of launch_equilibrium's size).  Starts and ends uniformly; the caller
// puts a barrier between two calls on the same workgroup (the LDS slab and flags are reused).
template <int BLOCK, bool INTEREST, int MODE = 0>
__device__ __forceinline__ void eq_column(const int b, const int j0, const int j1, const LearnBufs& L,
                                          const double* __restrict__ eta, const double* __restrict__ t_end,
                                          const double* __restrict__ u, const EqArgs& a, const InterestArgs& ia,
                                          const ResultSoA& out, double* smem)
{
    const int n = L.n_knots[b], ntau = L.n_tau[b], nle = L.n_le[b];
    const uint32_t lst = L.status[b];
    const size_t row = (size_t)b * (size_t)L.cap;
    const double* __restrict__ gT = L.t + row;
    const double* __restrict__ gG = L.G + row;
    const double* __restrict__ gH = L.hr + row;
    // Baseline: t and G staged (HR is read once per point by the blocked crossing scan, from
    // L2, with its block summaries in LDS) so that two workgroups fit a CU's LDS; the
    // interest mode stages HR too (its value functions look it up every RK stage).
    constexpr int NS = INTEREST ? 3 : 2;
    const bool fits = n <= a.lds_cap && (!INTEREST || ntau <= a.lds_cap);
    // MODE 1: the columns whose knots fit the LDS slab, MODE 2: the others, MODE 0: both.  The
    // sweeps launch 1 then 2, so the hot kernel carries no copy of the global-memory path (half
    // the machine code, no VGPR spills); a MODE-2 workgroup of a fitting column exits at once.
    if ((MODE == 1 && !fits) || (MODE == 2 && fits)) return;
    double* sT = smem;
    double* sG = smem + a.lds_cap;
    double* sH = INTEREST ? smem + 2 * a.lds_cap : nullptr;
    const double* __restrict__ cH = INTEREST ? sH : gH;
    // block summaries behind the three knot arrays (lds_cap/64 + 1 entries each)
    const int nsum = (a.lds_cap >> 6) + 1, nsum8 = (a.lds_cap >> 3) + 1;
    double* hmax = smem + NS * a.lds_cap;
    double* hmin = hmax + nsum;
    double* pmc = hmin + nsum;
    double* smc = pmc + nsum8;
    double* hpm = smc + nsum8; // crossing-scan tables (launch_equilibrium sizes the slab for them)
    double* hpn = hpm + nsum;
    double* hsm = hpn + nsum;
    double* hsn = hsm + nsum;
    const int nbh_s = (ntau + 63) >> 6;
    __shared__ int eq_next;
    __shared__ int s_nonmono;
    __shared__ int s_noscan;
    __shared__ int s_near1;                // two consecutive knots within 1e-15·t[n−1]
    __shared__ int s_ndec;                 // decreases of G between consecutive knots
    __shared__ unsigned long long s_maxdec; // largest decrease (bits of a nonnegative double)
    __shared__ double s_thalf;
    // every shared flag is initialised before the first barrier: lanes >= nq set
    // s_nonmono right after it, so a later store by thread 0 could clear their flag
    if (threadIdx.x == 0) { eq_next = 0; s_nonmono = 0; s_noscan = 0; s_near1 = 0; s_ndec = 0; s_maxdec = 0; s_thalf = NAN; }
    if (fits) {
        for (int i = threadIdx.x; i < n; i += BLOCK) { sT[i] = gT[i]; sG[i] = gG[i]; }
        if (INTEREST)
            for (int i = threadIdx.x; i < ntau; i += BLOCK) sH[i] = gH[i];
    }
    __syncthreads();
    Summ S{nullptr, nullptr, nullptr, nullptr, false, (double)NAN, false, 0.0, false, 2, nullptr, nullptr, nullptr,
           nullptr, 0};
    if (fits && !a.exhaustive) {
        const int nbh = (ntau + 63) >> 6, nbg = (n + 7) >> 3;
        // HR summaries: 8 lanes per 64-entry block, 8 independent loads each (HR is read from
        // L2), combined across the 8 lanes; then one lane per 8-knot G block
        const int nq = nbh << 3;
        for (int bk = threadIdx.x; bk < nq + nbg; bk += BLOCK) {
            if (bk < nq) {
                double mx = -INFINITY, mn = INFINITY;
                const int i0 = bk << 3;
                double h[8];
#pragma unroll
                for (int k = 0; k < 8; k++) h[k] = i0 + k < ntau ? cH[i0 + k] : -INFINITY;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    if (i0 + k >= ntau) continue;
                    if (h[k] > mx) mx = h[k];                                 // NaN never > u: ignore it
                    mn = (h[k] != h[k]) ? -INFINITY : (h[k] < mn ? h[k] : mn); // NaN is "not above"
                }
#pragma unroll
                for (int off = 1; off < 8; off <<= 1) { // the 8 lanes of a block are aligned in one wave
                    const double omx = __shfl_xor(mx, off, 8), omn = __shfl_xor(mn, off, 8);
                    mx = omx > mx ? omx : mx;
                    mn = omn < mn ? omn : mn;
                }
                if ((bk & 7) == 0) {
                    hmax[bk >> 3] = mx;
                    hmin[bk >> 3] = mn;
                }
            } else {
                const int g = bk - nq;
                double mx = -INFINITY, mn = INFINITY;
                const int e = (g << 3) + 8 < n ? (g << 3) + 8 : n;
                double prev = g > 0 ? sG[(g << 3) - 1] : -INFINITY;
                bool mono = true, nan = false;
                int ndec = 0;
                double maxdec = 0.0;
                for (int i = g << 3; i < e; i++) {
                    const double v = sG[i];
                    if (v != v) { mx = NAN; mn = NAN; mono = false; nan = true; break; }
                    if (v > mx) mx = v;
                    if (v < mn) mn = v;
                    const bool dec = v < prev;
                    mono &= !dec;
                    ndec += dec ? 1 : 0;
                    maxdec = dec && prev - v > maxdec ? prev - v : maxdec;
                    prev = v;
                }
                if (!mono) s_nonmono = 1;
                if (nan) s_noscan = 1;
                if (ndec) {
                    atomicAdd(&s_ndec, ndec);
                    atomicMax(&s_maxdec, (unsigned long long)sbr_dbits(maxdec));
                }
                // aw_scan's knot separation (Summ::scan)
                const double sep = 1e-15 * sT[n - 1];
                bool far = true, far1 = true;
                for (int i = g << 3; i < e; i++) {
                    far &= i + 2 >= n || sT[i + 2] - sT[i] > sep;
                    far1 &= i + 1 >= n || sT[i + 1] - sT[i] > sep;
                }
                if (!far) s_noscan = 1;
                if (!far1) s_near1 = 1;
                pmc[g] = mx; // block max for now
                smc[g] = mn; // block min for now
            }
        }
        __syncthreads();
        // prefix max / suffix min over blocks (NaN-propagating), two waves at once
        if (threadIdx.x == 0) {
            // t_half: first knot interval with G[k] <= 1/2 < G[k+1] (heuristic only)
            int lo = 0, hi = n - 1;
            if (n >= 2 && sG[0] <= 0.5 && sG[n - 1] > 0.5) {
                while (hi - lo > 1) {
                    const int mid = (lo + hi) >> 1;
                    if (sG[mid] <= 0.5) lo = mid;
                    else hi = mid;
                }
                s_thalf = sT[lo] + (0.5 - sG[lo]) * (sT[hi] - sT[lo]) / (sG[hi] - sG[lo]);
            }
            // the tables are read only when G is not monotone (Summ::mono) and aw_scan's
            // preconditions fail (the scan's points never read them): skip the serial scans
            if (s_nonmono && s_noscan)
            for (int g = 1; g < nbg; g++) {
                const double a0 = pmc[g - 1], b0 = pmc[g];
                pmc[g] = (a0 != a0 || b0 != b0) ? NAN : (a0 > b0 ? a0 : b0);
            }
        } else if (threadIdx.x == (BLOCK > 64 ? 64 : 1) && s_nonmono && s_noscan) {
            for (int g = nbg - 2; g >= 0; g--) {
                const double a0 = smc[g + 1], b0 = smc[g];
                smc[g] = (a0 != a0 || b0 != b0) ? NAN : (a0 < b0 ? a0 : b0);
            }
        }
        // the crossing scans' prefix / suffix tables over the HR blocks (hmax has no NaN, hmin has
        // NaN as −∞): a wave each way, 64 blocks per shuffle scan; small blocks: one lane each way
        if (BLOCK >= 256 && (threadIdx.x >> 6) >= 2 && (threadIdx.x >> 6) <= 3) {
            const bool fwd = (threadIdx.x >> 6) == 2;
            const int ln = threadIdx.x & 63;
            double ca = -INFINITY, cb = INFINITY;
            for (int c0 = 0; c0 < nbh; c0 += 64) {
                const int g = fwd ? c0 + ln : nbh - 1 - c0 - ln;
                const bool in = fwd ? g < nbh : g >= 0;
                double a = in ? hmax[g] : -INFINITY, b = in ? hmin[g] : INFINITY;
                for (int off = 1; off < 64; off <<= 1) {
                    const double oa = __shfl_up(a, off, 64), ob = __shfl_up(b, off, 64);
                    if (ln >= off) { a = oa > a ? oa : a; b = ob < b ? ob : b; }
                }
                a = ca > a ? ca : a;
                b = cb < b ? cb : b;
                if (in) {
                    if (fwd) { hpm[g] = a; hpn[g] = b; }
                    else { hsm[g] = a; hsn[g] = b; }
                }
                ca = __shfl(a, 63, 64);
                cb = __shfl(b, 63, 64);
            }
        }
        if (BLOCK < 256 && threadIdx.x == 2) {
            double a0 = -INFINITY, b0 = INFINITY;
            for (int g = 0; g < nbh; g++) {
                a0 = hmax[g] > a0 ? hmax[g] : a0;
                b0 = hmin[g] < b0 ? hmin[g] : b0;
                hpm[g] = a0;
                hpn[g] = b0;
            }
        }
        if (BLOCK < 256 && threadIdx.x == 3) {
            double a0 = -INFINITY, b0 = INFINITY;
            for (int g = nbh - 1; g >= 0; g--) {
                a0 = hmax[g] > a0 ? hmax[g] : a0;
                b0 = hmin[g] < b0 ? hmin[g] : b0;
                hsm[g] = a0;
                hsn[g] = b0;
            }
        }
        __syncthreads();
        const double dd = (double)s_ndec * sbr_bitsd(s_maxdec); // ≥ the largest drawdown
        S = Summ{hmax, hmin, pmc, smc, s_nonmono == 0, s_thalf,
                 n >= 2 && !s_noscan && dd <= 1e-12 && sG[0] >= 0.0 && sG[n - 1] <= 2.0, dd,
                 s_nonmono == 0 || s_noscan != 0, s_near1 == 0 ? 1 : 2,
                 hpm, hpn, hsm, hsn, nbh_s};
    }
    // Points are handed out to waves 64 at a time from an LDS counter, so a
    // wave that drew cheap no-run points goes back for more instead of idling
    // at the end of the block while the run points (bisection + AW_max) of its
    // neighbours finish.  Consecutive u in one wave keep its lanes on similar
    // control paths (runs form a prefix in u on the paper's grids).
    const int lane = threadIdx.x & 63;
    const double ETA = eta[b], T1 = t_end[b];
    const uint32_t lbits = lst & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED | SBR_KNOT_OVERFLOW);
    const bool bad_col = (lst & (SBR_ARG_INVALID | SBR_OOB)) || n < 2;
    const bool trunc = !a.full_grid && n >= 2 && gT[n - 1] < T1;
    for (;;) {
        int base = 0;
        if (lane == 0) base = atomicAdd(&eq_next, 64);
        base = __builtin_amdgcn_readfirstlane(base);
        if (j0 + base >= j1) break;
        const int j = j0 + base + lane;
        if (j >= j1) continue;
        const double uj = u[j];
        PointResult r;
        int64_t vsteps = 0;
        if (bad_col || !(uj >= 0.0)) {
            r.xi = NAN; r.aw = NAN; r.tol = INFINITY; r.iters = 0;
            r.tin = NAN; r.tout = NAN;
            r.status = ((lst & SBR_ARG_INVALID) || !(uj >= 0.0)) ? SBR_ARG_INVALID : (SBR_OOB | lbits);
        } else if (INTEREST && ia.r > 0.0) {
            if (MODE != 2 && fits)
                solve_interest_point(sT, sG, sH, S, n, ntau, nle, ETA, T1, trunc, uj, a.kappa, a.max_iters, lbits, ia,
                                     r, vsteps, a.aw_path, a.diag);
            else if (MODE != 1)
                solve_interest_point(gT, gG, gH, S, n, ntau, nle, ETA, T1, trunc, uj, a.kappa, a.max_iters, lbits, ia,
                                     r, vsteps, a.aw_path, a.diag);
        } else if (MODE != 2 && fits) {
            solve_point((const double*)sT, (const double*)sG, cH, S, n, ntau, nle, ETA, T1, trunc, uj, a.kappa,
                        a.max_iters, lbits, r, a.aw_path, a.diag);
        } else if (MODE != 1) {
            solve_point(gT, gG, gH, S, n, ntau, nle, ETA, T1, trunc, uj, a.kappa, a.max_iters, lbits, r, a.aw_path, a.diag);
        }
        const size_t o = (size_t)b * (size_t)a.n_u + j;
        if (INTEREST && ia.steps) ia.steps[o] = vsteps;
        out.xi[o] = r.xi;
        out.tau_in_unc[o] = r.tin;
        out.tau_out_unc[o] = r.tout;
        out.aw_max[o] = r.aw;
        out.tol[o] = r.tol;
        out.status[o] = r.status;
        if (out.iters) out.iters[o] = r.iters;
    }
}

#ifdef SBR_EQ_WGTIME
// diagnostic build only (tools/wgtime.py): per-workgroup start / end (100 MHz realtime clock)
// and hardware ids of the last equilibrium_kernel launch
constexpr size_t kWgTimeMax = 65536;
__device__ unsigned long long g_wgtime[2 * kWgTimeMax];
__device__ unsigned int g_wghw[2 * kWgTimeMax];
#endif

template <int BLOCK, bool INTEREST, int MODE>
__global__ __launch_bounds__(BLOCK, INTEREST ? 1 : kEqMinW) void equilibrium_kernel(LearnBufs L, const double* __restrict__ eta,
                                                            const double* __restrict__ t_end,
                                                            const double* __restrict__ u, EqArgs a, InterestArgs ia,
                                                            ResultSoA out)
{
    extern __shared__ double smem[];
    int b = (int)blockIdx.y;
    if (a.group > 1) { // grouped launch: the copies of a column back to back
        const int per = (int)gridDim.y / a.group;
        b = (b % a.group) * per + b / a.group;
    }
    const int j0 = blockIdx.x * EQ_TILE;
    const int j1 = j0 + EQ_TILE < a.n_u ? j0 + EQ_TILE : a.n_u;
#ifdef SBR_EQ_WGTIME
    const unsigned long long wt0 = __builtin_amdgcn_s_memrealtime();
#endif
    eq_column<BLOCK, INTEREST, MODE>(b, j0, j1, L, eta, t_end, u, a, ia, out, smem);
#ifdef SBR_EQ_WGTIME
    __syncthreads();
    const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    if (threadIdx.x == 0 && wg < kWgTimeMax) {
        g_wgtime[2 * wg] = wt0;
        g_wgtime[2 * wg + 1] = __builtin_amdgcn_s_memrealtime();
        // HW_ID (SE / CU / SIMD of wave 0) and XCC_ID: where the workgroup ran
        g_wghw[2 * wg] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
        g_wghw[2 * wg + 1] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11));
    }
#endif
}

// ============================================================================
// Readiness sweep, equilibrium side: workgroups take (column, u-tile) items in the order the
// learning kernel publishes the columns (ReadyArgs), so that a column's equilibria start as
// soon as its own ODE is solved instead of after the slowest column of the grid.  The
// tile-0 taker runs the column's hazard_rate first.
// ============================================================================
// poll *p (acquire) until it is set; 0 after `limit` polls or once another workgroup has
// given up (*err set): a stuck schedule drains in one timeout, not one per workgroup
__device__ __forceinline__ int ready_wait(const int32_t* p, const int32_t* err, int limit)
{
    int v = 0;
    for (int k = 0; k < limit; k++) {
        v = __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (v) break;
        if ((k & 63) == 63 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        __builtin_amdgcn_s_sleep(8);
    }
    return v;
}

// One workgroup per item, n_items in the grid: a workgroup draws its item ticket when it
// starts (tickets follow the publication order, so resident workgroups wait for the columns
// that come next), rather than persistent workgroups looping over items — a loop around the
// equilibrium body lets the compiler hoist its invariants and spill the 80-VGPR budget.
__global__ __launch_bounds__(kEqWide, kEqMinW) void eq_ready_kernel(LearnBufs L, const double* __restrict__ beta,
                                                                            const double* __restrict__ eta,
                                                                            const double* __restrict__ t_end,
                                                                            const double* __restrict__ u, LearnArgs la,
                                                                            EqArgs a, ReadyArgs ra, ResultSoA out)
{
    extern __shared__ double smem[];
    __shared__ int s_col, s_tile;
    const InterestArgs none{0.0, 1.0, 0.0, 0.0, 0, nullptr, nullptr, nullptr};
    if (threadIdx.x == 0) {
        const int it = atomicAdd(ra.head, 1);
        int col = -1, tile = 0;
        if (it < ra.n_items) {
            const int slot = it / ra.tiles;
            tile = it - slot * ra.tiles;
            const int v = ready_wait(ra.q + slot, ra.head + 1, ra.spin_limit);
            col = v ? v - 1 : -2;
            if (col >= 0 && tile > 0 && !ready_wait(ra.hz_flag + col, ra.head + 1, ra.spin_limit)) col = -2;
        }
        s_col = col;
        s_tile = tile;
    }
    __syncthreads();
    const int col = __builtin_amdgcn_readfirstlane(s_col), tile = __builtin_amdgcn_readfirstlane(s_tile);
    if (col == -1) return;
    if (col == -2) { // gave up waiting (a bug guard): the grid still drains
        if (threadIdx.x == 0) atomicOr(ra.head + 1, 1);
        return;
    }
    if (tile == 0) {
        // (the LDS-chunked path: the register-resident one needs 5 × 16 doubles per thread,
        // which the equilibrium's 80-VGPR budget would spill)
        hazard_column<kEqWide, false>(col, beta[col], eta[col], la, L, smem, smem + (HZ_LDS + 1),
                                          smem + 2 * (HZ_LDS + 1), smem + 3 * HZ_LDS + 2);
        __syncthreads();
        if (threadIdx.x == 0 && ra.tiles > 1)
            __hip_atomic_store(ra.hz_flag + col, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    const int j0 = tile * ra.tile_u;
    const int j1 = j0 + ra.tile_u < a.n_u ? j0 + ra.tile_u : a.n_u;
    eq_column<kEqWide, false>(col, j0, j1, L, eta, t_end, u, a, none, out, smem);
}

// ============================================================================
// One point by a whole workgroup (sbr_equilibrium_on_knots / sbr_solve_point_paths with
// n_u = 1: the drop-in's per-u calls).  The throughput kernel gives each point one lane, so a
// lone point pays every dependent LDS round trip of its searches (≈12 per lookup, ≈4 lookups
// per bisection iteration) and its staging runs on one wave.  Here the knots are staged by
// the whole block, wave 0 runs the point with wave-wide searches — searchsortedlast over [lo,
// hi] by 64-ary probing: one LDS load per lane and a ballot per round, two rounds for a
// Fig 5 column — and the block evaluates get_AW on every τ̄ knot (the exhaustive path), so
// AW_max and the three paths come from one pass.  The same operations as solve_point /
// solve_from_buffers' exact iteration and eval_range (each lookup lands on the bracket
// ssl_range finds: the knots are sorted), so the same bits.
// ============================================================================
constexpr int CO_BLOCK = 256;

// searchsortedlast in [lo, hi] (ssl_range's result for sorted t: lo + #{j in (lo, hi] : t[j] <= x})
// by the 64 lanes of a wave; every lane returns the same index.  Call with the whole wave active.
template <class P>
__device__ __forceinline__ int wave_ssl(P t, int lo, int hi, double x)
{
    const int lane = threadIdx.x & 63;
    if (lo >= hi) return lo; // a one-knot bracket (most bisection iterates once narrowed)
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) >> 6; // probes lo + k·step, k = 1..64 (those <= hi)
        const int pk = lo + (lane + 1) * step;
        const bool pr = pk <= hi && t[pk <= hi ? pk : hi] <= x;
        const int c = __popcll(__ballot(pr)); // the true probes are a prefix (t sorted)
        const int nhi = lo + (c + 1) * step - 1;
        hi = nhi < hi ? nhi : hi;
        lo = lo + c * step;
    }
    const int pk = lo + 1 + lane;
    const bool pr = pk <= hi && t[pk <= hi ? pk : hi] <= x;
    return lo + __popcll(__ballot(pr));
}

// lane k's double (k wave-uniform)
__device__ __forceinline__ double co_rl(double x, int k)
{
    const uint64_t u = sbr_dbits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
    return sbr_bitsd(((uint64_t)hi << 32) | lo);
}

// wave-uniform in_range (the flag as solve_from_buffers sets it)
__device__ __forceinline__ bool co_in_range(double x, double tlo, double thi, bool trunc, uint32_t& flag)
{
    if (x >= tlo && x <= thi) return true;
    flag |= (trunc && x > thi) ? SBR_ENGINE_TRUNC : SBR_OOB;
    return false;
}

template <class P>
__device__ __forceinline__ void point_wave(P T, P G, P H, const int n, const int ntau, const int nle,
                                           const double ETA, const double T1, const bool trunc, const double u,
                                           const double kappa, const int max_iters, const uint32_t lbits,
                                           PointResult& r, const double guess)
{
    const int lane = threadIdx.x & 63;
    r.xi = NAN; r.aw = NAN; r.tol = INFINITY; r.iters = 0; r.status = 0;
    // ---------------- optimal_buffer (solver.jl:211-264), 64 τ̄ entries per round ----------------
    bool any = false, all = true;
    int fa = -1, la = -1, cin = -1, cout = -1;
    for (int b0 = 0; b0 < ntau; b0 += 64) {
        const int i = b0 + lane;
        const bool in = i < ntau;
        const bool ab = in && H[in ? i : 0] > u;
        const bool pv = in && i > 0 && H[i > 0 && in ? i - 1 : 0] > u;
        const unsigned long long mab = __ballot(ab), min_ = __ballot(in);
        any |= mab != 0ull;
        all &= (mab & min_) == min_;
        if (mab) {
            if (fa < 0) fa = b0 + __ffsll((long long)mab) - 1;
            la = b0 + 63 - __clzll((long long)mab);
        }
        const unsigned long long mi = __ballot(in && i > 0 && !pv && ab); // 0 → 1 at i: cin = i − 1
        const unsigned long long mo = __ballot(in && i > 0 && pv && !ab); // 1 → 0 at i: cout = i − 1
        if (cin < 0 && mi) cin = b0 + __ffsll((long long)mi) - 2;
        if (mo) cout = b0 + 63 - __clzll((long long)mo) - 1;
    }
    auto tau = [&](int i) -> double { return i < nle ? T[i] : ETA; };
    double tin, tout;
    if (!any) {
        tin = T1; tout = T1;
    } else if (all) {
        tin = tau(0); tout = tau(ntau - 1);
    } else {
        tin = T1; tout = T1;
        if (cin >= 0) {
            const double t0 = tau(cin), t1 = tau(cin + 1), h0 = H[cin], h1 = H[cin + 1];
            tin = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
        }
        if (cout >= 0) {
            const double t0 = tau(cout), t1 = tau(cout + 1), h0 = H[cout], h1 = H[cout + 1];
            tout = t0 + ((u - h0) * (t1 - t0)) / (h1 - h0);
        }
        if (tin == T1) tin = tau(fa);
        if (tout == T1) tout = tau(la);
    }
    r.tin = tin;
    r.tout = tout;
    const double tlo = T[0], thi = T[n - 1];
    if (tin == tout) {
        r.status = SBR_NO_RUN_HR_BELOW_U | SBR_CONVERGED | lbits;
        r.tol = 0.0;
        return;
    }
    // ---------------- compute_ξ (solver.jl:308-376): the exact iteration ----------------
    uint32_t flag = 0;
    const double tolerance = 10.0 * sbr_jl_eps(kappa);
    uint32_t s = SBR_NO_RUN_MAXITER;
    double xi = NAN, tolr = INFINITY;
    if (guess == guess) { // ξ_guess: the plain iteration (solve_from_buffers), wave-uniform
        bisect_plain(T, G, n, tlo, thi, trunc, tin, tout, guess, kappa, tolerance, max_iters, r, flag, s, xi, tolr);
    } else {
    double xnew = (tin + tout) / 2.0, xmin = tin, xmax = tout;
    const bool okmin = co_in_range(xmin, tlo, thi, trunc, flag);
    const bool okmax = co_in_range(xmax, tlo, thi, trunc, flag);
    if (!okmin || !okmax) { r.status = flag | lbits; return; }
    int jlo = wave_ssl(T, 0, n - 1, xmin);
    int jhi = wave_ssl(T, 0, n - 1, xmax);
    const int jtin = jlo;
    // Rounds of six bisection levels at once: lane ℓ < 63 evaluates node k = ℓ + 1 of the
    // depth-6 tree below the current state (heap order; child 2k follows err > 0, 2k + 1
    // err < 0), replaying its path's midpoint arithmetic exactly, then the wave walks the tree
    // with the nodes' signs.  Each node runs the serial iteration's tests in its order; the walk
    // stops at the first terminal node on the path — the iteration where the serial loop breaks,
    // with its counters, flags and (for |err| <= tol) the slope probe, done by the whole wave.
    int iter0 = 1;
    for (;;) {
        const int k = lane + 1;
        const int d = 31 - __builtin_clz(k);
        double nmin = xmin, nmax = xmax, xo = xnew;
        for (int b = d - 1; b >= 0; b--) {
            if (((k >> b) & 1) == 0) { nmax = xo; xo = 0.5 * (xo + nmin); }
            else { nmin = xo; xo = 0.5 * (xo + nmax); }
        }
        const int it = iter0 + d;
        int term = 0; // 1 collapse, 2 max_iters − 1, 3 range flag, 4 |err| <= tol, 5 past max_iters
        uint32_t nflag = 0;
        double err = 0.0, AW = 0.0, oc = 0.0, ic = 0.0, xoe = 0.0, xie = 0.0;
        int j = 0, joc = 0, jic = 0;
        bool oke = false, oki = false;
        if (lane < 63) {
            if (it > max_iters) term = 5;
            else if (collapsed(nmin - nmax)) term = 1;
            else if (it == max_iters - 1) term = 2;
            else {
                ic = dmin(tin, xo); oc = dmin(tout, xo);
                j = ssl_range(T, jlo, jhi, xo);
                const bool ok = co_in_range(oc, tlo, thi, trunc, nflag);
                joc = (oc == xo) ? j : (ok ? ssl_range(T, 0, n - 1, oc) : 0);
                const double Goc = ok ? lerp_at(T, G, n, joc, oc) : 0.0;
                double Gic = 0.0;
                if (co_in_range(ic, tlo, thi, trunc, nflag)) {
                    jic = (ic == tin) ? jtin : (ic == xo ? j : ssl_range(T, 0, n - 1, ic));
                    Gic = lerp_at(T, G, n, jic, ic);
                }
                if (j + 1 >= n) {
                    nflag |= trunc ? SBR_ENGINE_TRUNC : SBR_OOB;
                    term = 3;
                } else {
                    const double eps = T[j + 1] - T[j];
                    xoe = oc + eps; xie = ic + eps;
                    oke = co_in_range(xoe, tlo, thi, trunc, nflag);
                    oki = co_in_range(xie, tlo, thi, trunc, nflag);
                    if (nflag) term = 3;
                    else {
                        AW = Goc - Gic;
                        err = AW - kappa;
                        if (fabs(err) <= tolerance) term = 4;
                    }
                }
            }
        }
        int node = 1, stop = 0;
        for (int lev = 0; lev < 6 && !stop; lev++) {
            const int src = node - 1;
            const int t_ = __builtin_amdgcn_readlane(term, src);
            if (t_) {
                stop = 1;
                r.iters = t_ == 5 ? max_iters : iter0 + lev;
                if (t_ == 1) s = SBR_NO_RUN_COLLAPSE;
                else if (t_ == 2) s = SBR_NO_RUN_MAXITER;
                else if (t_ == 3) flag |= (uint32_t)__builtin_amdgcn_readlane((int)nflag, src);
                else if (t_ == 4) {
                    const double xo_t = co_rl(xo, src), AW_t = co_rl(AW, src), err_t = co_rl(err, src);
                    const double xoe_t = co_rl(xoe, src), xie_t = co_rl(xie, src);
                    const int joc_t = __builtin_amdgcn_readlane(joc, src), jic_t = __builtin_amdgcn_readlane(jic, src);
                    const bool oke_t = __builtin_amdgcn_readlane(oke ? 1 : 0, src) != 0;
                    const bool oki_t = __builtin_amdgcn_readlane(oki ? 1 : 0, src) != 0;
                    double Goce = 0.0, Gice = 0.0;
                    if (oke_t) Goce = lerp_at(T, G, n, wave_ssl(T, joc_t, n - 1, xoe_t), xoe_t);
                    if (oki_t) Gice = lerp_at(T, G, n, wave_ssl(T, jic_t, n - 1, xie_t), xie_t);
                    const double AWe = Goce - Gice;
                    if (AWe >= AW_t) { s = SBR_RUN; xi = xo_t; tolr = fabs(err_t); }
                    else s = SBR_FALSE_EQ;
                }
                break;
            }
            const double e_ = co_rl(err, src);
            const int j_ = __builtin_amdgcn_readlane(j, src);
            if (e_ > 0) jhi = j_; else jlo = j_;
            if (lev == 5) { // the next round's state: the child of this depth-5 node
                const double xs = co_rl(xo, src), mn = co_rl(nmin, src), mxv = co_rl(nmax, src);
                if (e_ > 0) { xmin = mn; xmax = xs; xnew = 0.5 * (xs + mn); }
                else { xmin = xs; xmax = mxv; xnew = 0.5 * (xs + mxv); }
            }
            node = 2 * node + (e_ > 0 ? 0 : 1);
        }
        if (stop) break;
        iter0 += 6;
    }
    } // default first iterate
    if (flag) { r.status = flag | lbits; return; }
    if (s != SBR_RUN) { r.status = s | lbits; return; }
    // the AW stage's own range checks (solve_from_buffers: G(0), then the path's last τ̄ — the
    // shifted arguments are nondecreasing, so the first failing knot fails there too)
    if (!co_in_range(0.0, tlo, thi, trunc, flag)) { r.status = flag | lbits; return; }
    const double icc = (tin >= xi) ? xi : tin;
    const double occ = (tout > xi) ? xi : tout;
    const double al = (tau(ntau - 1) - xi) + icc, bl = (tau(ntau - 1) - xi) + occ;
    if (!((al > 0 ? al : 0.0) <= thi) || !((bl > 0 ? bl : 0.0) <= thi)) {
        r.status = (trunc ? SBR_ENGINE_TRUNC : SBR_OOB) | lbits;
        return;
    }
    r.xi = xi;
    r.tol = tolr;
    r.status = SBR_RUN | SBR_CONVERGED | lbits; // r.aw: the block's get_AW pass
}

// get_AW on τ̄ entries [i0, i1) with brackets slid along (eval_range's arithmetic); NaN-latching
// max into mx (Julia maximum), paths written when given
template <class P>
__device__ __forceinline__ void co_eval(P T, P G, const int n, const int nle, const double ETA, const double xi,
                                        const double icc, const double occ, const double G0, const int i0,
                                        const int i1, double& mx, double* __restrict__ aw_cum,
                                        double* __restrict__ aw_out, double* __restrict__ aw_in)
{
    if (i0 >= i1) return;
    auto tau = [&](int i) -> double { return i < nle ? T[i] : ETA; };
    auto x_of = [&](int i, double c) { const double v = (tau(i) - xi) + c; return v > 0 ? v : 0.0; };
    int ka = ssl_range(T, 0, n - 1, x_of(i0, icc)), kb = ssl_range(T, 0, n - 1, x_of(i0, occ));
    ka = ka < n - 2 ? ka : n - 2;
    kb = kb < n - 2 ? kb : n - 2;
    double ta0 = T[ka], ta1 = T[ka + 1], ga0 = G[ka], ga1 = G[ka + 1];
    double tb0 = T[kb], tb1 = T[kb + 1], gb0 = G[kb], gb1 = G[kb + 1];
    for (int i = i0; i < i1; i++) {
        const double ti = tau(i);
        const double av = (ti - xi) + icc;
        const double bv = (ti - xi) + occ;
        const double xa = av > 0 ? av : 0.0;
        const double xb = bv > 0 ? bv : 0.0;
        while (ka < n - 2 && ta1 <= xa) { ka++; ta0 = ta1; ga0 = ga1; ta1 = T[ka + 1]; ga1 = G[ka + 1]; }
        while (kb < n - 2 && tb1 <= xb) { kb++; tb0 = tb1; gb0 = gb1; tb1 = T[kb + 1]; gb1 = G[kb + 1]; }
        const double da = (xa - ta0) / (ta1 - ta0);
        const double gi = ga0 * (1.0 - da) + ga1 * da;
        double go;
        if (xb == tb0) go = gb0 * 1.0 + gb1 * 0.0; // eval_range's δ = 0 form (the same value)
        else { const double db = (xb - tb0) / (tb1 - tb0); go = gb0 * (1.0 - db) + gb1 * db; }
        const double awin = av >= 0 ? gi : 0.0;
        const double awout = bv >= 0 ? go : 0.0;
        const double v = (awout - awin) + G0;
        if (aw_cum) aw_cum[i] = v;
        if (aw_out) aw_out[i] = awout;
        if (aw_in) aw_in[i] = awin;
        if (mx == mx && (v != v || v > mx)) mx = v;
    }
}

__global__ __launch_bounds__(CO_BLOCK) void point_coop_kernel(LearnBufs L, const double* __restrict__ eta,
                                                              const double* __restrict__ t_end,
                                                              const double* __restrict__ u, EqArgs a, ResultSoA out)
{
    extern __shared__ double smem[];
    __shared__ double s_r[5];
    __shared__ uint32_t s_st;
    __shared__ int s_it;
    __shared__ double s_mx[CO_BLOCK / 64];
    const int n = L.n_knots[0], ntau = L.n_tau[0], nle = L.n_le[0];
    const uint32_t lst = L.status[0];
    const bool fits = n <= a.lds_cap && ntau <= a.lds_cap;
    double* sT = smem;
    double* sG = smem + a.lds_cap;
    double* sH = smem + 2 * a.lds_cap;
    if (fits) {
        for (int i = threadIdx.x; i < n; i += CO_BLOCK) { sT[i] = L.t[i]; sG[i] = L.G[i]; }
        for (int i = threadIdx.x; i < ntau; i += CO_BLOCK) sH[i] = L.hr[i];
    }
    __syncthreads();
    const double* T = fits ? (const double*)sT : (const double*)L.t;
    const double* G = fits ? (const double*)sG : (const double*)L.G;
    const double* H = fits ? (const double*)sH : (const double*)L.hr;
    // one workgroup per u value (a ξ_guess call over n_u values; paths only with one workgroup)
    const int jb = blockIdx.x;
    const double ETA = eta[0], T1 = t_end[0], uj = u[jb];
    const uint32_t lbits = lst & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED | SBR_KNOT_OVERFLOW);
    const bool bad_col = (lst & (SBR_ARG_INVALID | SBR_OOB)) || n < 2;
    const bool trunc = !a.full_grid && n >= 2 && L.t[n - 1] < T1;
    if (threadIdx.x < 64) {
        PointResult r;
        if (bad_col || !(uj >= 0.0)) {
            r.xi = NAN; r.aw = NAN; r.tol = INFINITY; r.iters = 0; r.tin = NAN; r.tout = NAN;
            r.status = ((lst & SBR_ARG_INVALID) || !(uj >= 0.0)) ? SBR_ARG_INVALID : (SBR_OOB | lbits);
        } else {
            point_wave(T, G, H, n, ntau, nle, ETA, T1, trunc, uj, a.kappa, a.max_iters, lbits, r, a.xi_guess);
        }
        if (threadIdx.x == 0) {
            s_r[0] = r.xi; s_r[1] = r.tin; s_r[2] = r.tout; s_r[3] = r.aw; s_r[4] = r.tol;
            s_st = r.status;
            s_it = r.iters;
        }
    }
    __syncthreads();
    const uint32_t st = s_st;
    double mx = -INFINITY;
    if (st & SBR_RUN) {
        const double xi = s_r[0], tin = s_r[1], tout = s_r[2];
        const double icc = (tin >= xi) ? xi : tin;
        const double occ = (tout > xi) ? xi : tout;
        const double G0 = lerp_at(T, G, n, ssl_range(T, 0, n - 1, 0.0), 0.0);
        // contiguous τ̄ ranges per thread (the brackets slide), a NaN-latching max per thread
        const int per = (ntau + CO_BLOCK - 1) / CO_BLOCK;
        const int i0 = threadIdx.x * per, i1 = i0 + per < ntau ? i0 + per : ntau;
        double* sc = a.path_scratch;
        if (sc && a.aw_path)
            co_eval(T, G, n, nle, ETA, xi, icc, occ, G0, i0, i1, mx, sc, a.aw_out_path ? sc + ntau : nullptr,
                    a.aw_in_path ? sc + 2 * ntau : nullptr);
        else
            co_eval(T, G, n, nle, ETA, xi, icc, occ, G0, i0, i1, mx, a.aw_path, a.aw_out_path, a.aw_in_path);
        // block reduction in thread order (NaN latches: any NaN gives NaN, else the max)
        for (int off = 32; off >= 1; off >>= 1) {
            const double o = __shfl_down(mx, off, 64);
            mx = (mx != mx || o != o) ? (double)NAN : (o > mx ? o : mx);
        }
        if ((threadIdx.x & 63) == 0) s_mx[threadIdx.x >> 6] = mx;
    }
    __syncthreads();
    if ((st & SBR_RUN) && a.path_scratch && a.aw_path) {
        // the rows formed per thread in scratch, copied out with consecutive lanes on consecutive
        // entries (a mapped-host destination then takes whole-line writes)
        const double* sc = a.path_scratch;
        for (int i = threadIdx.x; i < ntau; i += CO_BLOCK) {
            a.aw_path[i] = sc[i];
            if (a.aw_out_path) a.aw_out_path[i] = sc[ntau + i];
            if (a.aw_in_path) a.aw_in_path[i] = sc[2 * ntau + i];
        }
    }
    if (threadIdx.x == 0) {
        double aw = s_r[3];
        if (st & SBR_RUN) {
            aw = s_mx[0];
            for (int w = 1; w < CO_BLOCK / 64; w++) aw = (aw != aw || s_mx[w] != s_mx[w]) ? (double)NAN : (s_mx[w] > aw ? s_mx[w] : aw);
        }
        out.xi[jb] = s_r[0];
        out.tau_in_unc[jb] = s_r[1];
        out.tau_out_unc[jb] = s_r[2];
        out.aw_max[jb] = aw;
        out.tol[jb] = s_r[4];
        out.status[jb] = st;
        if (out.iters) out.iters[jb] = s_it;
    }
}

hipError_t launch_point_coop(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                             const EqArgs& a, const ResultSoA& out, hipStream_t s, int n_points)
{
    if (n_points > 1 && (a.aw_path || a.aw_out_path || a.aw_in_path || a.path_scratch)) return hipErrorInvalidValue;
    const size_t lds = (size_t)3 * a.lds_cap * sizeof(double);
    hipLaunchKernelGGL(point_coop_kernel, dim3(n_points), dim3(CO_BLOCK), lds, s, L, eta, t_end, u, a, out);
    return hipGetLastError();
}

// ============================================================================
// launchers
// ============================================================================
hipError_t launch_learn_kernel(const double* beta, const double* eta, const double* t_end, const LearnArgs& a,
                               const LearnBufs& L, hipStream_t s, int mode)
{
    const unsigned waves = (unsigned)((a.n_beta + 63) / 64);
    // heads first: whole grids of one-wave blocks only
    if (a.wpg && (mode == 0 || a.wpg < 2 || a.head < 1 || a.head >= a.wpg || a.n_beta % (64 * a.wpg) != 0))
        return hipErrorInvalidValue;
    if (mode == 2) { // LDS-staged rows with the fused hazard (launch_hazard_norm after)
        if (!a.fuse_hazard) return hipErrorInvalidValue;
        hipLaunchKernelGGL((learn_logistic_kernel<64, true>), dim3(waves), dim3(64), kStageLdsPerWave, s,
                           beta, eta, t_end, a, L);
    } else if (mode == 0) {
        hipLaunchKernelGGL(learn_logistic_kernel<kLearnBlock>, dim3((a.n_beta + kLearnBlock - 1) / kLearnBlock),
                           dim3(kLearnBlock), 0, s, beta, eta, t_end, a, L);
    } else {
        static_assert(kLearnBlockLat == 64, "mode 1 runs one-wave blocks");
        hipLaunchKernelGGL(learn_logistic_kernel<kLearnBlockLat>, dim3(waves), dim3(kLearnBlockLat), 0, s, beta, eta,
                           t_end, a, L);
    }
    return hipGetLastError();
}

hipError_t launch_hazard_norm(const LearnArgs& a, const LearnBufs& L, int n_cols, hipStream_t s)
{
    hipLaunchKernelGGL(hazard_norm_kernel, dim3(n_cols), dim3(HN_BLOCK), 0, s, a, L);
    return hipGetLastError();
}

hipError_t launch_learn_logistic(const double* beta, const double* eta, const double* t_end, const LearnArgs& a,
                                 const LearnBufs& L, hipStream_t s)
{
    hipError_t e = launch_learn_kernel(beta, eta, t_end, a, L, s, (a.fuse_hazard && !a.ready_q) ? 0 : 1);
    if (e != hipSuccess) return e;
    if (a.ready_q) return hipSuccess; // readiness sweep: eq_ready_kernel runs each column's hazard
    if (a.fuse_hazard) return launch_hazard_norm(a, L, a.n_beta, s);
    hipLaunchKernelGGL(hazard_kernel, dim3(a.n_beta), dim3(HZ_BLOCK), 0, s, beta,
                       eta, a, L);
    return hipGetLastError();
}

hipError_t launch_hazard(const double* beta, const double* eta, const LearnArgs& a, const LearnBufs& L, int n_beta,
                         hipStream_t s)
{
    hipLaunchKernelGGL(hazard_kernel, dim3(n_beta), dim3(HZ_BLOCK), 0, s, beta, eta, a, L);
    return hipGetLastError();
}

hipError_t launch_equilibrium(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                              const EqArgs& a, const ResultSoA& out, int n_beta, hipStream_t s, int only_mode)
{
    const size_t lds = ((size_t)2 * a.lds_cap + 6 * ((a.lds_cap >> 6) + 1) + 2 * ((a.lds_cap >> 3) + 1)) * sizeof(double);
    // one block per (β column, tile of EQ_TILE u values); block size by tile width.  Wide
    // tiles use 12-wave blocks: two per CU (LDS holds two columns' t and G) = 6 waves/SIMD.
    const int tiles = (a.n_u + EQ_TILE - 1) / EQ_TILE;
    const int w = a.n_u < EQ_TILE ? a.n_u : EQ_TILE;
    dim3 grid(tiles, n_beta);
    const InterestArgs none{0.0, 1.0, 0.0, 0.0, 0, nullptr, nullptr, nullptr};
    // the LDS-resident columns, then (a workgroup per column, exiting at once where it fits, no
    // LDS slab) the columns beyond the slab on the global-memory path
    auto go = [&](auto k1, auto k2, int bs) {
        if (only_mode != 2) hipLaunchKernelGGL(k1, grid, dim3(bs), lds, s, L, eta, t_end, u, a, none, out);
        if (only_mode != 1) hipLaunchKernelGGL(k2, grid, dim3(bs), 0, s, L, eta, t_end, u, a, none, out);
    };
    if (w > 256)
        go(equilibrium_kernel<kEqWide, false, 1>, equilibrium_kernel<kEqWide, false, 2>, kEqWide);
    else if (w > 64)
        go(equilibrium_kernel<256, false, 1>, equilibrium_kernel<256, false, 2>, 256);
    else
        go(equilibrium_kernel<64, false, 1>, equilibrium_kernel<64, false, 2>, 64);
    return hipGetLastError();
}

hipError_t launch_eq_ready(const LearnBufs& L, const double* beta, const double* eta, const double* t_end,
                           const double* u, const LearnArgs& la, const EqArgs& a, const ReadyArgs& ra,
                           const ResultSoA& out, int n_blocks, hipStream_t s)
{
    size_t lds = ((size_t)2 * a.lds_cap + 6 * ((a.lds_cap >> 6) + 1) + 2 * ((a.lds_cap >> 3) + 1)) * sizeof(double);
    const size_t hz = (size_t)(3 * HZ_LDS + 3) * sizeof(double); // hazard scratch shares the slab
    if (lds < hz) lds = hz;
    (void)n_blocks; // one workgroup per item
    hipLaunchKernelGGL(eq_ready_kernel, dim3(ra.n_items), dim3(kEqWide), lds, s, L, beta, eta, t_end, u, la, a, ra,
                       out);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void ready_fail_kernel(const int32_t* __restrict__ gave_up, ResultSoA out,
                                                          int64_t n_pts)
{
    if (__hip_atomic_load(gave_up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_pts; i += (int64_t)gridDim.x * 256) {
        out.xi[i] = NAN;
        out.tau_in_unc[i] = NAN;
        out.tau_out_unc[i] = NAN;
        out.aw_max[i] = NAN;
        out.tol[i] = INFINITY;
        out.status[i] = SBR_ENGINE_SCHED;
        if (out.iters) out.iters[i] = 0;
    }
}

hipError_t launch_ready_fail(const int32_t* gave_up, const ResultSoA& out, int64_t n_pts, hipStream_t s)
{
    hipLaunchKernelGGL(ready_fail_kernel, dim3(256), dim3(256), 0, s, gave_up, out, n_pts);
    return hipGetLastError();
}

hipError_t launch_interest(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                           const EqArgs& a, const InterestArgs& ia, const ResultSoA& out, int n_beta, hipStream_t s)
{
    const size_t lds = ((size_t)3 * a.lds_cap + 6 * ((a.lds_cap >> 6) + 1) + 2 * ((a.lds_cap >> 3) + 1)) * sizeof(double);
    // every lane integrates its own value function (~5·10⁴ Tsit5 steps): one wave per 64 u
    // of the column so that all of them run at once (the LDS slab allows one block per CU)
    const int tiles = (a.n_u + EQ_TILE - 1) / EQ_TILE;
    const int w = a.n_u < EQ_TILE ? a.n_u : EQ_TILE;
    dim3 grid(tiles, n_beta);
    auto go = [&](auto k1, auto k2, int bs) {
        hipLaunchKernelGGL(k1, grid, dim3(bs), lds, s, L, eta, t_end, u, a, ia, out);
        hipLaunchKernelGGL(k2, grid, dim3(bs), 0, s, L, eta, t_end, u, a, ia, out);
    };
    if (w > 512)
        go(equilibrium_kernel<1024, true, 1>, equilibrium_kernel<1024, true, 2>, 1024);
    else if (w > 256)
        go(equilibrium_kernel<512, true, 1>, equilibrium_kernel<512, true, 2>, 512);
    else if (w > 64)
        go(equilibrium_kernel<256, true, 1>, equilibrium_kernel<256, true, 2>, 256);
    else
        go(equilibrium_kernel<64, true, 1>, equilibrium_kernel<64, true, 2>, 64);
    return hipGetLastError();
}

}  // namespace sbr

#ifdef SBR_EQ_WGTIME
// diagnostic build only: copy the workgroup timeline of the last equilibrium launch (n entries)
extern "C" int sbr_diag_wgtime_read(unsigned long long* t2, unsigned int* hw2, int n)
{
    if (n < 0 || (size_t)n > sbr::kWgTimeMax) return -1;
    if (hipMemcpyFromSymbol(t2, HIP_SYMBOL(sbr::g_wgtime), sizeof(unsigned long long) * 2 * n) != hipSuccess) return -2;
    if (hipMemcpyFromSymbol(hw2, HIP_SYMBOL(sbr::g_wghw), sizeof(unsigned int) * 2 * n) != hipSuccess) return -2;
    return 0;
}
#endif
