// sbr_social.hip — gfx950 kernels for the social-learning extension sweep:
// every (β, u) point runs the fixed point of solve_equilibrium_social_learning
// (src/extensions/social_learning/social_learning_solver.jl:63-263):
//
//   AW_0 = G of the baseline SI learning on (0, η)               (:89-94)
//   repeat  G_n  = Tsit5 solve of dG/dt = (1 − G) β AW_{n−1}(t)   (dynamics.jl:58-78)
//           r_n  = solve_equilibrium_baseline on G_n              (:139-143)
//           AW*  = get_AW(ξ_n or ξ_{n−1} + η/500, …) on G_n        (:147-200)
//           stop if ‖AW* − AW_{n−1}‖_∞ on range(0, η, 1000) < tol  (:162-172, :195-212)
//           AW_n = ½ AW_{n−1} + ½ AW* on G_n's knots              (:174-178, :218-222)
//
// Layout and schedule:
//  * one lane per grid point for the whole fixed point — the forced ODE is a
//    serial chain of ~10⁵ Tsit5 steps per iterate, so points are the only
//    parallelism; lanes of a wave hold consecutive u of one β column;
//  * each point owns five knot buffers of `cap` doubles in HBM (wave-blocked,
//    see BView): AW_{n−1} knots/values, G_n knots, values and AW_{n−1}(t_i) at
//    those knots; buffers rotate between iterates;
//  * a point whose iterate outgrows `cap` moves into a promotion pool of 16×
//    the capacity and redoes that iterate there (pool blocks of the same launch);
//  * one launch per fixed-point iterate over a worklist of unfinished points;
//    a single-workgroup ballot compaction (order-preserving, deterministic)
//    retires finished lanes so later iterates launch only live waves.
//
// Bit-exact against oracle/sbr_oracle.c social_point (same operation order,
// -ffp-contract=off, fma() where the oracle has it, shared sbr_exp/sbr_log).
#include <type_traits>

#include "sbr_device.h"
#include "sbr_kernels.h"
#include "sbr_ode.h"

namespace sbr {

namespace {

// One point's knot buffer in the wave-blocked layout: 16 consecutive knots of a
// point fill one 128-byte line, and the 64 points of a wave group interleave
// line by line (an 8 KiB row per 16-knot block).  A lane still streams its own
// lines sequentially, but a wave's 64 concurrent accesses fall within a few
// MiB instead of 64 separate multi-MiB rows (page/TLB locality).
// Typed address spaces (A/B knob): the workspace is global memory and the rings are LDS.  With
// generic pointers the compiler issues FLAT loads, and it merges a ring read and its global
// fallback (`in_ring ? RT(j) : to[j]`) into one FLAT load of a selected pointer; a FLAT load
// counts on both the vector-memory and the LDS counters, so every ring read waited for the
// lane's outstanding global loads and stores.
typedef double sbr_dv2 __attribute__((ext_vector_type(2))); // 16-byte knot pair
typedef __attribute__((address_space(1))) double gdouble;
typedef __attribute__((address_space(1))) char gchar;
typedef __attribute__((address_space(1))) sbr_dv2 gdouble2;
typedef __attribute__((address_space(3))) double ldouble;
struct BView {
    gdouble* p; // ws + (group·5 + slot)·cap·64 + lane·16
    // 32-bit byte offset (a group's buffer is < 4 GiB): one shift-and-or pair, no sign extension
    __device__ __forceinline__ gdouble& operator[](int k) const
    {
        const uint32_t u = (uint32_t)k;
        return *(gdouble*)((gchar*)p + (((u >> 4) << 13) | ((u & 15u) << 3)));
    }
};

// Bracket search with an 8-knot window of knot times held in registers: the
// walks below advance a few knots per lookup, so brackets come from register
// compares and only the interpolation operands are loaded (independent loads,
// no dependent search chains).  Returns exactly searchsortedlast's index.
struct Win8 {
    BView t;
    int n;
    int wb;        // window base: tw[k] = t[wb + k] (+Inf past the grid)
    double tw[8];
    // branch-free refill: eight independent loads (index clamped into the grid)
    __device__ __forceinline__ void load(int base)
    {
        wb = base;
        const int last = n > 0 ? n - 1 : 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int i = base + k;
            const double v = t[i < last ? i : last];
            tw[k] = (i < n) ? v : (double)INFINITY;
        }
    }
    __device__ __forceinline__ void init(BView tt, int nn)
    {
        t = tt;
        n = nn;
        load(0);
    }
    __device__ int slow_find(double x) const
    {
        return (x >= tw[0]) ? ssl_gallop(t, n, wb + 7, x) : ssl_range(t, 0, wb, x);
    }
    // largest j with t[j] <= x; requires t[0] <= x; the window does not move
    __device__ __forceinline__ int find(double x) const
    {
        int c = 0;
#pragma unroll
        for (int k = 1; k < 7; k++) c += (tw[k] <= x) ? 1 : 0;
        int j = wb + c;
        if (!(x >= tw[0] && x < tw[7])) j = slow_find(x);
        return j;
    }
    // same, then re-centre the window on the answer once it is 4+ knots ahead
    __device__ __forceinline__ int find_advance(double x)
    {
        const int j = find(x);
        if (j - wb >= 4 || j < wb) load(j);
        return j;
    }
};

// gridded-linear value on bracket j (clamped to [0, n-2]) with unconditional
// loads, NaN + oob when x is outside [t_0, t_{n-1}] (oracle interp_s)
__device__ __forceinline__ double lerp_sel(BView t, BView v, int n, int j, double x, bool in)
{
    j = j > n - 2 ? n - 2 : j;
    j = j < 0 ? 0 : j;
    const double t0 = t[j], t1 = t[j + 1], v0 = v[j], v1 = v[j + 1];
    const double d = (x - t0) / (t1 - t0);
    const double r = v0 * (1.0 - d) + v1 * d;
    return in ? r : (double)NAN;
}

// Interpolations.jl gridded Linear with Throw() (oracle interp_s): NaN + oob
// outside [t_0, t_{n-1}].  Monotone walker over one knot grid.
struct Walker {
    Win8 w;
    BView v;
    double tfirst, tlast;
    __device__ __forceinline__ void init(BView tt, BView vv, int nn)
    {
        w.init(tt, nn);
        v = vv;
        tfirst = nn > 0 ? tt[0] : 0.0;
        tlast = nn > 0 ? tt[nn - 1] : 0.0;
    }
    __device__ __forceinline__ double at(double x, bool& oob)
    {
        const bool in = w.n >= 2 && x >= tfirst && x <= tlast;
        oob |= !in;
        const int j = in ? w.find_advance(x) : 0;
        return lerp_sel(w.t, v, w.n, j, x, in);
    }
    // bracket only (clamped like lerp_at); requires t[0] <= x <= t[n-1]
    __device__ __forceinline__ int bracket(double x)
    {
        const int j = w.find_advance(x);
        return j > w.n - 2 ? w.n - 2 : j;
    }
};


// A ring miss loads its operands from global memory inside a divergent branch.  Unless the
// branch waits for them itself, the wait lands where the ring path writes the same registers,
// and it is a vmcnt wait that also drains every older store and refill load of the wave — on
// every lookup, whether or not any lane missed.  vmcnt(0) here (expcnt/lgkmcnt left alone)
// is paid only when a lane misses.
__device__ __forceinline__ void ring_miss_wait()
{
    __builtin_amdgcn_s_waitcnt(0x0F70);
}

// knots k, k+1 (k even) of one lane in one 16-byte load: a pair never straddles a 16-knot line
__device__ __forceinline__ double2 ld2(BView b, int k)
{
    const uint32_t u = (uint32_t)k;
    const sbr_dv2 v = *(const gdouble2*)((const gchar*)b.p + (((u >> 4) << 13) | ((u & 15u) << 3)));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st2(BView b, int k, double x, double y)
{
    const uint32_t u = (uint32_t)k;
    *(gdouble2*)((gchar*)b.p + (((u >> 4) << 13) | ((u & 15u) << 3))) = sbr_dv2{x, y};
}

// Walker with the knot values held beside the knot times: an 8-knot window on a 4-aligned base,
// filled by four paired loads per array, so both bracket and interpolation operands come from
// registers (one refill per ~4 knots of walk instead of 4 operand loads per lookup).  Same
// brackets and the same lerp_at arithmetic as Walker.
struct WalkerV {
    BView t, v;
    int n, wb;
    double tw[8], vw[8];
    double tfirst, tlast;
    __device__ __forceinline__ void load(int base)
    {
        wb = base;
        const int q = n > 0 ? ((n - 1) & ~1) : 0; // last pair that holds a knot (k+1 < cap: cap is a multiple of 16)
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int k = base + 2 * m;
            const int kc = k < q ? k : q;
            const double2 a = ld2(t, kc), b = ld2(v, kc);
            tw[2 * m] = (k < n) ? a.x : (double)INFINITY;
            tw[2 * m + 1] = (k + 1 < n) ? a.y : (double)INFINITY;
            vw[2 * m] = b.x;
            vw[2 * m + 1] = b.y;
        }
    }
    __device__ __forceinline__ void init(BView tt, BView vv, int nn)
    {
        t = tt;
        v = vv;
        n = nn;
        load(0);
        tfirst = nn > 0 ? tw[0] : 0.0;
        tlast = nn > 0 ? tt[nn - 1] : 0.0;
    }
    __device__ __forceinline__ int find_advance(double x)
    {
        int c = 0;
#pragma unroll
        for (int k = 1; k < 7; k++) c += (tw[k] <= x) ? 1 : 0;
        int j = wb + c;
        if (!(x >= tw[0] && x < tw[7]))
            j = (x >= tw[0]) ? ssl_gallop(t, n, wb + 7, x) : ssl_range(t, 0, wb, x);
        if (j - wb >= 4 || j < wb) load(j & ~3);
        return j;
    }
    __device__ __forceinline__ static double sel4(const double* w, int r)
    {
        const double lo = (r & 1) ? w[1] : w[0];
        const double hi = (r & 1) ? w[3] : w[2];
        return (r & 2) ? hi : lo;
    }
    __device__ __forceinline__ double at(double x, bool& oob)
    {
        const bool in = n >= 2 && x >= tfirst && x <= tlast;
        oob |= !in;
        if (!in) return (double)NAN;
        int j = find_advance(x);
        j = j > n - 2 ? n - 2 : j;
        j = j < 0 ? 0 : j;
        const int r = j - wb;
        double t0, t1, v0, v1;
        if (r >= 0 && r < 4) {
            t0 = sel4(tw, r); t1 = sel4(tw + 1, r);
            v0 = sel4(vw, r); v1 = sel4(vw + 1, r);
        } else { // x == t_{n-1} on a window that starts at n−1
            t0 = t[j]; t1 = t[j + 1]; v0 = v[j]; v1 = v[j + 1];
            ring_miss_wait();
        }
        const double d = (x - t0) / (t1 - t0);
        return v0 * (1.0 - d) + v1 * d;
    }
};

// full-range lookup (non-monotone callers: the bisection)
__device__ __forceinline__ double interp_full(BView t, BView v, int n, double x, bool& oob)
{
    if (n < 2 || !(x >= t[0] && x <= t[n - 1])) { oob = true; return (double)NAN; }
    return lerp_at(t, v, n, ssl_range(t, 0, n - 1, x), x);
}

__device__ __forceinline__ BView buf_at(double* ws, int cap, int l, int slot)
{
    return BView{(gdouble*)(ws + ((size_t)(l >> 6) * 5 + (size_t)slot) * (size_t)cap * 64 + (size_t)(l & 63) * 16)};
}
__device__ __forceinline__ BView buf(const SocialArgs& a, int l, int slot) { return buf_at(a.ws, a.cap, l, slot); }

// Move a point whose iterate outgrew the knot capacity into a pool slot with
// its state from before that iterate (AW_{n-1}, ξ, status bits, step count);
// the pool blocks of this or the next launch redo the iterate.  False when
// the pool is full (the point then retires with SBR_KNOT_OVERFLOW and the
// host re-runs it at a larger capacity).
__device__ bool promote(const SocialArgs& a, int l, int64_t g, int iter, BView TO, BView VO, int n_old)
{
    const SocialPool& q = a.pool;
    if (n_old > q.cap) return false;
    const int s = atomicAdd(q.used, 1);
    if (s >= q.n_slots) return false;
    BView BT = buf_at(q.ws, q.cap, s, 0), BV = buf_at(q.ws, q.cap, s, 1);
    for (int i = 0; i < n_old; i++) {
        BT[i] = TO[i];
        BV[i] = VO[i];
    }
    q.n_old[s] = n_old;
    q.slots[s] = 0u | (1u << 3) | (2u << 6) | (3u << 9) | (4u << 12);
    q.xi_new[s] = a.xi_new[l];
    q.bits[s] = a.bits[l];
    q.steps[s] = a.steps[l];
    q.live[s] = 1;
    q.pts[s] = g;
    q.it_cur[s] = iter;
    atomicAdd(q.n_live, 1);
    __hip_atomic_store(q.ready + s, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    a.live[l] = 0;
    return true;
}


// ---- one point on all 64 lanes (COOP): the streaming passes over the point's knots, by chunks
// of 64 consecutive knots (lane L holds knot c0 + L).  The per-knot work is done lane-parallel;
// only the trapezoid sum is a serial fold, taken in the reference's order (I = I + term_i, i
// ascending, every term formed exactly as the serial loop forms it), so every value is the
// serial loop's bit for bit.  One memory round trip per 64 knots instead of one per knot.
__device__ __forceinline__ double rl_d(double x, int k)
{
    const uint64_t u = sbr_dbits(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
    return sbr_bitsd(((uint64_t)hi << 32) | lo);
}
// lane L gets lane L − 1's value, lane 0 gets `first`
__device__ __forceinline__ double up_d(double x, double first)
{
    const double v = __shfl_up(x, 1, 64);
    return (threadIdx.x & 63) == 0 ? first : v;
}

// hazard_rate on τ̄ = the knots (solver.jl:153-185) and optimal_buffer's crossing scan
// (:211-264): the two passes of social_iterate's serial path.  X receives exp(λ t_i) and IA the
// running integral I_i (scratch buffers of the point).
__device__ void coop_hazard_scan(BView T, BView Gv, BView AWO, BView X, BView IA, const int n, const double BETA,
                                 const double lam, const double p, const double U, const double ETA, bool& any,
                                 bool& all, int& first_above, int& last_above, double& tin_c, double& tout_c)
{
    const int L = (int)(threadIdx.x & 63);
    const double omp = 1.0 - p;
    // pass A: e_i = exp(λ t_i)·pdf_i, term_i = (0.5·(e_{i−1} + e_i))·(t_i − t_{i−1}), I_i = I_{i−1} + term_i
    double I = 0.0, ec = 0.0, tc = 0.0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int i = c0 + L;
        const bool v = i < n;
        const int ix = v ? i : n - 1;
        const double ti = T[ix];
        const double ex = sbr_exp(lam * ti);
        if (v) X[i] = ex;
        const double e = ex * (((1.0 - Gv[ix]) * BETA) * AWO[ix]);
        const double ep = up_d(e, ec), tp = up_d(ti, tc);
        const double term = (0.5 * (ep + e)) * (ti - tp);
        const int m = n - c0 < 64 ? n - c0 : 64;
        double Ii = 0.0;
        for (int k = 0; k < m; k++) {
            if (c0 + k > 0) I = I + rl_d(term, k);
            Ii = L == k ? I : Ii;
        }
        if (v) IA[i] = Ii;
        ec = rl_d(e, 63);
        tc = rl_d(ti, 63);
    }
    const double Ieta = I;
    // pass B: HR_i = ((p·X_i)·pdf_i)/((p·I_i) + (1 − p)·I_η) and the crossings with u
    bool have_in = false;
    double hc = 0.0;
    tc = 0.0;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int i = c0 + L;
        const bool v = i < n;
        const int ix = v ? i : n - 1;
        const double ti = T[ix];
        const double pdf = ((1.0 - Gv[ix]) * BETA) * AWO[ix];
        const double hr = ((p * X[ix]) * pdf) / ((p * IA[ix]) + (omp * Ieta));
        const double hp = up_d(hr, hc), tp = up_d(ti, tc);
        const bool ab = v && hr > U, abp = hp > U;
        const uint64_t mv = __ballot(v), mab = __ballot(ab);
        const uint64_t mrise = __ballot(v && i >= 1 && !abp && ab), mfall = __ballot(v && i >= 1 && abp && !ab);
        any |= mab != 0;
        all &= mab == mv;
        if (mab) {
            if (first_above < 0) first_above = c0 + __builtin_ctzll(mab);
            last_above = c0 + 63 - __builtin_clzll(mab);
        }
        const double cross = tp + ((U - hp) * (ti - tp)) / (hr - hp);
        if (!have_in && mrise) {
            tin_c = rl_d(cross, __builtin_ctzll(mrise));
            have_in = true;
        }
        if (mfall) tout_c = rl_d(cross, 63 - __builtin_clzll(mfall));
        hc = rl_d(hr, 63);
        tc = rl_d(ti, 63);
    }
}

// searchsortedlast(T, x) for T[0] <= x from a per-lane hint (either side of the answer)
__device__ __forceinline__ int coop_ssl(BView T, int n, int hint, double x) { return ssl_near(T, n, hint, x); }

// the damping AW_n(t_i) = ½ AW_{n−1}(t_i) + ½ AW*(t_i) on G_n's knots (social_learning_solver.jl
// :174-178, :218-222) with AW* = get_AW(ξ, …) evaluated as aw_at does — lane-parallel: lane L
// evaluates AW* at knot c0 + L (its own bracket searches, hinted by its previous chunk) and
// damps knot c0 + L − 1, whose interpolation weights need AW* at both knots.
__device__ void coop_damping(BView T, BView Gv, BView AWO, const int n, const double XI, const double ic,
                             const double oc, const double G0, bool& aoob)
{
    const int L = (int)(threadIdx.x & 63);
    const double tfirst = T[0], tlast = T[n - 1];
    int ha = 0, hb = 0;
    double awc = 0.0;
    bool bad = false;
    for (int c0 = 0; c0 < n; c0 += 64) {
        const int i = c0 + L;
        const bool v = i < n;
        const int ix = v ? i : n - 1;
        const double tau = T[ix];
        const double xa = (tau - XI) + ic, xb = (tau - XI) + oc;
        const double xa0 = xa > 0 ? xa : 0.0, xb0 = xb > 0 ? xb : 0.0;
        const bool ina = n >= 2 && xa0 >= tfirst && xa0 <= tlast;
        const bool inb = n >= 2 && xb0 >= tfirst && xb0 <= tlast;
        bad |= v && !(ina && inb);
        ha = ina ? coop_ssl(T, n, ha, xa0) : ha;
        hb = inb ? coop_ssl(T, n, hb, xb0) : hb;
        const double gi = lerp_sel(T, Gv, n, ina ? ha : 0, xa0, ina);
        const double go = lerp_sel(T, Gv, n, inb ? hb : 0, xb0, inb);
        const double awin = xa >= 0 ? gi : 0.0;
        const double awout = xb >= 0 ? go : 0.0;
        const double aw = (awout - awin) + G0;
        const double awm = up_d(aw, awc);
        if (v && i >= 1) {
            const double vn = awm * (1.0 - 0.0) + aw * 0.0;
            AWO[i - 1] = 0.5 * AWO[i - 1] + 0.5 * vn;
        }
        if (v && i == n - 1) {
            const double vl = awm * (1.0 - 1.0) + aw * 1.0;
            AWO[n - 1] = 0.5 * AWO[n - 1] + 0.5 * vl;
        }
        awc = rl_d(aw, 63);
        ha += 64;
        hb += 64;
    }
    aoob |= __ballot(bad) != 0;
}


constexpr int kRing = 64; // knots per lane: four 16-knot lines (two lines per lane for 64 lanes was slower: r04_z)

constexpr int kRingLanes = 32; // lanes a multi-point wave may use (the launch makes L <= this)
constexpr size_t kRingLdsBytes = (size_t)2 * kRing * kRingLanes * sizeof(double); // t and v: 32 KiB either way

// dG/dt = (1 − G) β AW_old(t) (social_learning_dynamics.jl:61-67) for a wave that runs many
// points (the bulk of a sweep: up to 32 per wave).  All stage times of a step (t + c_i·dt,
// t + dt) are known when the step starts, so the five AW_old lookups are done up front
// (prepare), off the serial chain of the RK stages.  Every lane streams its own knot lines, so each operand load of a stage lookup is a separate
// L1 request per active lane: ≈25 load instructions per RK step × 32 lanes, and the L1 cannot
// hold 4 waves × 32 lanes × the lines in use (PMC of the bulk: 66 % of wave cycles waiting on
// memory, against 40 % for a lone point, profiles/r04_pmc_social_bulk_vs_lone.txt).  Here each
// lane keeps AW_{n−1}'s knots [rb, rb + 32) (times and values) in a ring in LDS, layout
// [slot][lane] (slot = knot mod 32): a lookup's four operands are LDS reads; the ring advances
// by one 128-byte line (16 knots, eight 16-byte loads per array) when the accepted time's
// bracket passes rb + 20, and the line after next is touched into L2 then.  The bracket window
// (Win8) reloads from the ring too.  Knots outside the ring fall back to global loads.  Same
// brackets, operands and operations as the oracle's forced right-hand side: bit-identical.
struct SocialRhsRing {
    double beta;
    BView to;
    BView vo;
    int n;
    double tfirst, tlast;
    Win8 w;
    double aw[5];
    double last_aw;
    bool oob;
    int slow;
    ldouble* rt; // this lane's ring: rt[s * kRingLanes] = t[k] for the knot k ≡ s (mod 32) held
    ldouble* rv;
    int rb;     // first knot held (a multiple of 16)
    int tick = 0; // attempted Tsit5 steps (prepare calls): equal across the live lanes of a wave
    double pf_t = 0.0, pf_v = 0.0;
    static constexpr bool kAcceptFirst = true; // refill before the knot's stores (ode_scalar)
    __device__ __forceinline__ bool in_ring(int j) const { return j >= rb && j + 1 < rb + kRing; }
    __device__ __forceinline__ double RT(int j) const { return rt[(j & (kRing - 1)) * kRingLanes]; }
    __device__ __forceinline__ double RV(int j) const { return rv[(j & (kRing - 1)) * kRingLanes]; }
    // knots [base, base + 16) into their slots (base a multiple of 16; nothing past the grid)
    __device__ __forceinline__ void fill_line(int base)
    {
        if (base >= n) return;
        const gdouble2* lt = (const gdouble2*)((const gchar*)to.p + ((size_t)(base >> 4) << 13));
        const gdouble2* lv = (const gdouble2*)((const gchar*)vo.p + ((size_t)(base >> 4) << 13));
        sbr_dv2 a[8], b[8];
#pragma unroll
        for (int q = 0; q < 8; q++) { a[q] = lt[q]; b[q] = lv[q]; }
        const int s0 = base & (kRing - 1);
#pragma unroll
        for (int q = 0; q < 8; q++) {
            rt[(s0 + 2 * q) * kRingLanes] = a[q].x; rt[(s0 + 2 * q + 1) * kRingLanes] = a[q].y;
            rv[(s0 + 2 * q) * kRingLanes] = b[q].x; rv[(s0 + 2 * q + 1) * kRingLanes] = b[q].y;
        }
    }
    // Win8's refill with the ring's copies where it holds them
    __device__ __forceinline__ void wload(int base)
    {
        w.wb = base;
        const int last = n > 0 ? n - 1 : 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int i = base + k;
            const int ic = i < last ? i : last;
            double v;
            if (ic >= rb && ic < rb + kRing) v = RT(ic);
            else { v = to[ic]; ring_miss_wait(); }
            w.tw[k] = (i < n) ? v : (double)INFINITY;
        }
    }
    __device__ __forceinline__ int find_advance(double x)
    {
        const int j = w.find(x);
        if (j - w.wb >= 4 || j < w.wb) wload(j);
        return j;
    }
    // lerp_sel with the operands from the ring where it holds them
    __device__ __forceinline__ double lerp_r(int j, double x, bool in) const
    {
        j = j > n - 2 ? n - 2 : j;
        j = j < 0 ? 0 : j;
        double t0, t1, v0, v1;
        if (in_ring(j)) { t0 = RT(j); t1 = RT(j + 1); v0 = RV(j); v1 = RV(j + 1); }
        else { t0 = to[j]; t1 = to[j + 1]; v0 = vo[j]; v1 = vo[j + 1]; ring_miss_wait(); }
        const double d = (x - t0) / (t1 - t0);
        const double r = v0 * (1.0 - d) + v1 * d;
        return in ? r : (double)NAN;
    }
    __device__ __forceinline__ void init(double b, BView t_, BView v_, int n_, double* ring)
    {
        slow = 0;
        beta = b; to = t_; vo = v_; n = n_;
        tfirst = n > 0 ? to[0] : 0.0;
        tlast = n > 0 ? to[n - 1] : 0.0;
        oob = false;
        last_aw = 0.0;
        const int lane = (int)(threadIdx.x & 63);
        rt = (ldouble*)ring + lane;
        rv = (ldouble*)ring + kRing * kRingLanes + lane;
        rb = 0;
#pragma unroll
        for (int b = 0; b < kRing; b += 16) fill_line(b);
        w.t = to;
        w.n = n;
        wload(0);
    }
    __device__ __forceinline__ double lookup(double x)
    {
        if (n < 2 || !(x >= tfirst && x <= tlast)) { oob = true; return (double)NAN; }
        return lerp_r(w.find(x), x, true);
    }
    __device__ __forceinline__ double eval(double t, double x)
    {
        const double a = lookup(t);
        last_aw = a;
        return ((1.0 - x) * beta) * a;
    }
    __device__ __forceinline__ void prepare(double t, double dt)
    {
        tick++;
        const double xs[5] = {fma(C1, dt, t), fma(C2, dt, t), fma(C3, dt, t), fma(C4, dt, t), t + dt};
        int js[5];
        bool in[5];
#pragma unroll
        for (int k = 0; k < 5; k++) {
            in[k] = n >= 2 && xs[k] >= tfirst && xs[k] <= tlast;
            slow += (in[k] && !(xs[k] < w.tw[7])) ? 1 : 0;
            js[k] = w.find(in[k] ? xs[k] : tfirst);
        }
#pragma unroll
        for (int k = 0; k < 5; k++) {
            aw[k] = lerp_r(js[k], xs[k], in[k]);
            oob |= !in[k];
        }
        last_aw = aw[4];
    }
    __device__ __forceinline__ double stage(int s, double, double x) const
    {
        return ((1.0 - x) * beta) * aw[s < 5 ? s - 1 : 4];
    }
    __device__ __forceinline__ void jac(double t, double x, double& J, double& dT)
    {
        if (n < 2 || !(t >= tfirst && t <= tlast)) {
            oob = true;
            J = (double)NAN;
            dT = (double)NAN;
            return;
        }
        int j = w.find(t);
        j = j > n - 2 ? n - 2 : (j < 0 ? 0 : j);
        double t0, t1, v0, v1;
        if (in_ring(j)) { t0 = RT(j); t1 = RT(j + 1); v0 = RV(j); v1 = RV(j + 1); }
        else { t0 = to[j]; t1 = to[j + 1]; v0 = vo[j]; v1 = vo[j + 1]; ring_miss_wait(); }
        const double d = (t - t0) / (t1 - t0);
        const double a = v0 * (1.0 - d) + v1 * d;
        const double rr = 1.0 / (t1 - t0);
        const double ap = v0 * (-rr) + v1 * rr;
        J = ((-1.0) * beta) * a;
        dT = ((1.0 - x) * beta) * ap;
    }
    __device__ __forceinline__ void accepted(double t)
    {
        if (n >= 2 && t >= tfirst && t <= tlast) {
            const int j = find_advance(t);
            // Four lines: a lane whose bracket has passed rb + 20 replaces its oldest lines
            // (wb > j − 4 >= the new rb), but only on every 8th attempted step — the same step
            // for every lane of the wave, so one wave-wide wait on the refill loads serves all
            // the lanes due — unless fewer than 24 knots are left ahead of the bracket.
            if (j + 2 >= rb + kRing) { // past the ring: re-seat it around j
                rb = ((j - 4) >> 4) << 4;
#pragma unroll
                for (int b = 0; b < kRing; b += 16) fill_line(rb + b);
            } else if (j - rb >= 20 && ((tick & 7) == 0 || j - rb >= kRing - 24)) {
                for (int k = 0; k < 3 && j - rb >= 20; k++) {
                    fill_line(rb + kRing);
                    rb += 16;
                }
                slow += (pf_t == -1.0 || pf_v == -2.0) ? 1 : 0;
                const int q = rb + kRing + 16 < n ? rb + kRing + 16 : n - 1;
                pf_t = to[q];
                pf_v = vo[q];
            }
        }
    }
    static constexpr bool kFsalExact = false;
    static constexpr bool kPinTableau = true;
};

// The same right-hand side for a wave whose 64 lanes all run ONE point (the tail of a sweep,
// when the spread worklist leaves one live point per wave): every lane executes the identical
// chain, and AW_{n−1}'s knots are held across the wave — lane L holds knot wb + L (time and
// value) — so a stage lookup is a ballot over the window (the lanes whose knot time is ≤ x form
// a prefix: the bracket is wb + popcount − 1) and four v_readlanes, instead of waiting on an
// L2/HBM round trip per step.  The window moves forward by 32 knots when the step's time passes
// its middle (one coalesced load per array); lookups outside it fall back to the global search.
// Same brackets, same operands, same operations as SocialRhsRing: bit-identical.
struct SocialRhsCoop {
    double beta;
    BView to;
    BView vo;
    int n;
    double tfirst, tlast;
    int wb;           // window base (wave-uniform)
    double wt, wv;    // this lane's knot wb + lane (+Inf / 0 past the grid)
    double aw[5];
    double last_aw;
    bool oob;
    int slow;
    __device__ __forceinline__ void refill(int base)
    {
        wb = base;
        const int i = base + (int)(threadIdx.x & 63);
        const int ic = i < n - 1 ? i : (n > 0 ? n - 1 : 0);
        const double t = to[ic], v = vo[ic];
        wt = i < n ? t : (double)INFINITY;
        wv = i < n ? v : 0.0;
    }
    __device__ __forceinline__ void init(double b, BView t_, BView v_, int n_)
    {
        slow = 0;
        beta = b; to = t_; vo = v_; n = n_;
        tfirst = n > 0 ? to[0] : 0.0;
        tlast = n > 0 ? to[n - 1] : 0.0;
        oob = false;
        last_aw = 0.0;
        refill(0);
    }
    __device__ __forceinline__ static double lane_d(double x, int k)
    {
        const uint64_t u = sbr_dbits(x);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, k);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), k);
        return sbr_bitsd(((uint64_t)hi << 32) | lo);
    }
    // searchsortedlast(t, x) for t[0] <= x <= t[n−1] (wave-uniform x)
    __device__ __forceinline__ int find(double x)
    {
        const int c = __popcll(__ballot(wt <= x));
        if (c >= 1 && c < 64) return wb + c - 1;
        slow++;
        return c == 0 ? ssl_range(to, 0, wb, x) : ssl_gallop(to, n, wb + 63, x);
    }
    // lerp_at(to, vo, n, j, x) with the operands from the window where it holds them
    __device__ __forceinline__ double lerp_j(int j, double x)
    {
        j = j > n - 2 ? n - 2 : j;
        j = j < 0 ? 0 : j;
        const int k = __builtin_amdgcn_readfirstlane(j - wb);
        double t0, t1, v0, v1;
        if (k >= 0 && k < 63) {
            t0 = lane_d(wt, k); t1 = lane_d(wt, k + 1); v0 = lane_d(wv, k); v1 = lane_d(wv, k + 1);
        } else {
            t0 = to[j]; t1 = to[j + 1]; v0 = vo[j]; v1 = vo[j + 1];
            ring_miss_wait(); // not at the join: there it would drain the knot stores every lookup
        }
        const double d = (x - t0) / (t1 - t0);
        return v0 * (1.0 - d) + v1 * d;
    }
    __device__ __forceinline__ double lookup(double x)
    {
        if (n < 2 || !(x >= tfirst && x <= tlast)) { oob = true; return (double)NAN; }
        return lerp_j(find(x), x);
    }
    __device__ __forceinline__ double eval(double t, double x)
    {
        const double a = lookup(t);
        last_aw = a;
        return ((1.0 - x) * beta) * a;
    }
    // lane k's copy of x from lane `src` (ds_bpermute, 64-bit as two dwords)
    __device__ __forceinline__ static double perm_d(double x, int src)
    {
        const uint64_t u = sbr_dbits(x);
        const uint32_t lo = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)u);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)(uint32_t)(u >> 32));
        return sbr_bitsd(((uint64_t)hi << 32) | lo);
    }
    __device__ __forceinline__ void prepare(double t, double dt)
    {
        const double xs[5] = {fma(C1, dt, t), fma(C2, dt, t), fma(C3, dt, t), fma(C4, dt, t), t + dt};
        // The five stage lookups side by side (1): the stage times depend on
        // t and dt only, so their brackets are five ballots over the window, and lane k runs stage
        // k's lerp — the same operands and operations as lerp_j, hence the same bits — on the
        // window knots it fetches with ds_bpermute; the five values come back by readlane.  One
        // division and one lerp of wave time instead of five, off the serial RK chain.  Any
        // stage time off the grid or past the window's last interval takes the serial form.
        {
            bool fast = n >= 2;
#pragma unroll
            for (int k = 0; k < 5; k++) fast &= xs[k] >= tfirst && xs[k] <= tlast;
            if (fast) {
                const int lane = (int)(threadIdx.x & 63);
                int src = 0;
                double xl = xs[4];
#pragma unroll
                for (int k = 0; k < 5; k++) {
                    const int c = __popcll(__ballot(wt <= xs[k]));
                    // bracket j = wb + c − 1 (searchsortedlast), clamped to n − 2 as lerp_j does;
                    // window lane q = j − wb must hold both operand knots (q < 63)
                    int q = c - 1;
                    q = q > n - 2 - wb ? n - 2 - wb : q;
                    fast &= c >= 1 && c < 64 && q >= 0 && q < 63;
                    src = lane == k ? q : src;
                    xl = lane == k ? xs[k] : xl;
                }
                if (fast) {
                    const double t0 = perm_d(wt, src), t1 = perm_d(wt, src + 1);
                    const double v0 = perm_d(wv, src), v1 = perm_d(wv, src + 1);
                    const double d = (xl - t0) / (t1 - t0);
                    const double a = v0 * (1.0 - d) + v1 * d;
#pragma unroll
                    for (int k = 0; k < 5; k++) aw[k] = lane_d(a, k);
                    last_aw = aw[4];
                    return;
                }
                slow++;
            }
        }
#pragma unroll
        for (int k = 0; k < 5; k++) {
            const bool in = n >= 2 && xs[k] >= tfirst && xs[k] <= tlast;
            aw[k] = in ? lerp_j(find(xs[k]), xs[k]) : (double)NAN;
            oob |= !in;
        }
        last_aw = aw[4];
    }
    __device__ __forceinline__ double stage(int s, double, double x) const
    {
        return ((1.0 - x) * beta) * aw[s < 5 ? s - 1 : 4];
    }
    __device__ __forceinline__ void jac(double t, double x, double& J, double& dT)
    {
        if (n < 2 || !(t >= tfirst && t <= tlast)) {
            oob = true;
            J = (double)NAN;
            dT = (double)NAN;
            return;
        }
        int j = find(t);
        j = j > n - 2 ? n - 2 : (j < 0 ? 0 : j);
        const double t0 = to[j], t1 = to[j + 1], v0 = vo[j], v1 = vo[j + 1];
        const double d = (t - t0) / (t1 - t0);
        const double a = v0 * (1.0 - d) + v1 * d;
        const double rr = 1.0 / (t1 - t0);
        const double ap = v0 * (-rr) + v1 * rr;
        J = ((-1.0) * beta) * a;
        dT = ((1.0 - x) * beta) * ap;
    }
    // re-anchor the window 8 knots behind the accepted time once it passes the window's middle
    __device__ __forceinline__ void accepted(double t)
    {
        if (n >= 2 && t >= tfirst && t <= tlast) {
            const int c = __popcll(__ballot(wt <= t));
            if (c >= 40) refill(wb + c - 9);
        }
    }
    static constexpr bool kFsalExact = false;
    static constexpr bool kPinTableau = true;
    static constexpr bool kAcceptFirst = true; // the refill's loads ahead of the knot stores
};

}  // namespace

// ============================================================================
// init: baseline learning on (0, η) as AW_0 (social_learning_solver.jl:89-94)
// ============================================================================
__global__ __launch_bounds__(64) void social_init_kernel(SocialArgs a)
{
    const int l = blockIdx.x * 64 + threadIdx.x;
    if (l >= a.n_pts) return;
    const int64_t g = a.pts ? a.pts[l] : a.pt0 + l;
    const int b = (int)(g / a.n_u);
    const double BETA = a.beta[b], ETA = a.eta[b];
    BView T = buf(a, l, 0);
    BView V = buf(a, l, 1);
    int n = 0;
    uint32_t st = 0;
    LogisticSys f{BETA};
    struct Sink {
        BView T, V;
        int& n;
        int cap;
        uint32_t& st;
        __device__ __forceinline__ bool push(double t, double x)
        {
            if (n >= cap) { st |= SBR_KNOT_OVERFLOW; return false; }
            T[n] = t;
            V[n] = x;
            n++;
            return true;
        }
        __device__ __forceinline__ bool start(double t, double x) { return push(t, x); }
        __device__ __forceinline__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&, bool)
        {
            return acc ? push(tn, y1) : true;
        }
    } sink{T, V, n, a.cap, st};
    OdeOut o;
    ode_scalar(f, sink, ETA, a.x0, a.rtol, a.atol, a.maxiters, o);
    st |= o.status & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED);
    a.n_old[l] = n;
    a.slots[l] = 0u | (1u << 3) | (2u << 6) | (3u << 9) | (4u << 12);
    a.xi_new[l] = 0.0;
    a.bits[l] = st;
    a.steps[l] = o.naccept + o.nreject;
    a.work[l] = l;
    // SolvedModel before any iterate (oracle social_point's initial `out`)
    a.out.xi[g] = (double)NAN;
    a.out.tau_in_unc[g] = (double)NAN;
    a.out.tau_out_unc[g] = (double)NAN;
    a.out.aw_max[g] = (double)NAN;
    a.out.tol[g] = (double)INFINITY;
    a.out.status[g] = 0;
    if (a.out.iters) a.out.iters[g] = 0;
    if (a.fp_iters) a.fp_iters[g] = 0;
    if (st & SBR_KNOT_OVERFLOW) { // engine limit: the point cannot be represented
        a.out.status[g] = SBR_KNOT_OVERFLOW | SBR_SOCIAL_NOT_CONVERGED;
        if (a.steps_out) a.steps_out[g] = a.steps[l];
        a.live[l] = 0;
    } else {
        a.live[l] = 1;
    }
    if (l == 0) a.count[0] = a.n_pts;
}

// ============================================================================
// ============================================================================
// one fixed-point iterate of point l (local index into a's per-point state);
// false once the point has finished or moved into the promotion pool
// ============================================================================
// COOP: all 64 lanes of the wave run this same point (SocialRhsCoop); every lane computes the
// same values and stores them to the same places, and the few non-idempotent steps (the pool
// promotion, the live counter) are taken by lane 0 alone.
template <bool COOP>
__device__ __forceinline__ bool social_iterate(const SocialArgs& a, int l, int iter, double* ring)
{
    const int64_t g = a.pts ? a.pts[l] : a.pt0 + l;
    const int b = (int)(g / a.n_u);
    const int ju = (int)(g % a.n_u);
    const double BETA = a.beta[b], ETA = a.eta[b], U = a.u[ju];
    const gdouble* __restrict__ CMP = (const gdouble*)(a.cmp + (size_t)b * a.n_cmp);
    const uint32_t P = a.slots[l];
    const int s_to = P & 7, s_vo = (P >> 3) & 7, s_t = (P >> 6) & 7, s_G = (P >> 9) & 7, s_aw = (P >> 12) & 7;
    BView TO = buf(a, l, s_to);
    BView VO = buf(a, l, s_vo);
    BView T = buf(a, l, s_t);
    BView Gv = buf(a, l, s_G);
    BView AWO = buf(a, l, s_aw);
    gdouble* CMPO = (gdouble*)(a.cmpo + (size_t)l * a.n_cmp);
    const int n_old = a.n_old[l];
    uint32_t bits = a.bits[l];
    const double xi_old = a.xi_new[l];

    // diagnostics: per-phase shader cycles (SBR_FLAG_DIAG_SOCIAL_PROF)
    int64_t* PR = a.prof ? a.prof + (size_t)l * 8 : nullptr;
    int64_t c0 = PR ? (int64_t)clock64() : 0;
    auto stamp = [&](int k) {
        if (PR) { const int64_t c1 = (int64_t)clock64(); PR[k] += c1 - c0; c0 = c1; }
    };
    // AW_{n-1} on the comparison grid, needed after its buffers are recycled
    bool cmp_oob = false;
    {
        Walker wo;
        wo.init(TO, VO, n_old);
        for (int k = 0; k < a.n_cmp; k++) CMPO[k] = wo.at(CMP[k], cmp_oob);
    }

    stamp(0);
    // ---- (a) learning from withdrawals on (0, η) ----
    typename std::conditional<COOP, SocialRhsCoop,
                              SocialRhsRing>::type f;
    if constexpr (!COOP) f.init(BETA, TO, VO, n_old, ring);
    else { (void)ring; f.init(BETA, TO, VO, n_old); }
    int n = 0;
    bool overflow = false;
    // knots (t, G) and AW_{n−1} at each knot: the t + dt stage lookup unless the step
    // was snapped to T1 (the first knot: AW_{n−1}(0))
    struct Sink {
        decltype(f)& f;
        BView T, Gv, AWO;
        int& n;
        int cap;
        bool& overflow;
        __device__ __forceinline__ bool push(double t, double x, double aw)
        {
            if (n >= cap) { overflow = true; return false; }
            T[n] = t;
            Gv[n] = x;
            AWO[n] = aw;
            n++;
            return true;
        }
        __device__ __forceinline__ bool start(double t, double x) { return push(t, x, f.lookup(t)); }
        __device__ __forceinline__ bool step(bool acc, double, double tn, double, double, double y1, const StepK&,
                                             bool exact)
        {
            if (!acc) return true;
            return push(tn, y1, exact ? f.last_aw : f.lookup(tn));
        }
    } sink{f, T, Gv, AWO, n, a.cap, overflow};
    OdeOut o;
    ode_scalar(f, sink, ETA, a.x0, a.rtol, a.atol, a.maxiters, o);
    stamp(1);
    if (PR) { PR[6] += f.slow; PR[7] += o.naccept + o.nreject; }
    if (f.oob) o.status |= SBR_OOB;
    if (overflow && a.pool.ws) {
        bool moved;
        if constexpr (COOP) {
            moved = false;
            if ((threadIdx.x & 63) == 0) moved = promote(a, l, g, iter, TO, VO, n_old);
            moved = __builtin_amdgcn_readfirstlane(moved ? 1 : 0) != 0;
        } else {
            moved = promote(a, l, g, iter, TO, VO, n_old);
        }
        if (moved) return false;
    }
    a.steps[l] += o.naccept + o.nreject;
    bits |= o.status & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED);

    bool finish = false, converged = false, stop_oob = false, need_awmax = false;
    double xi_r = (double)NAN, tin = (double)NAN, tout = (double)NAN, tol_r = (double)INFINITY;
    uint32_t st_r = 0;
    int32_t it_r = 0;
    bool have_r = false;
    double xi_n = xi_old;

    if (overflow) {
        finish = true;
        bits |= SBR_KNOT_OVERFLOW;
        stop_oob = false;
    } else if (o.status & SBR_OOB) {
        finish = true;
        stop_oob = true; // previous iterate's SolvedModel stays in `out`
    } else {
        have_r = true;
        if (a.path_aw && n <= a.path_cap) // before the damping below overwrites AW_{n-1}(t_i)
            for (int i = 0; i < n; i++) a.path_aw[i] = AWO[i];
        // ---- hazard_rate (solver.jl:153-185) on τ̄ = knots (t_n = η, else the η
        // append needs pdf(η) past the grid: BoundsError) ----
        const bool h_oob = !(n >= 2 && T[n - 1] == ETA);
        if (h_oob) {
            st_r = SBR_OOB;
        } else {
            BView X = TO; // AW_{n-1} knots are dead now: exp(λτ̄) scratch
            const double lam = a.lam, p = a.p, omp = 1.0 - p;
            bool any = false, all = true;
            int first_above = -1, last_above = -1;
            double tin_c = ETA, tout_c = ETA;
            bool have_in = false;
            if constexpr (COOP) {
                coop_hazard_scan(T, Gv, AWO, X, VO, n, BETA, lam, p, U, ETA, any, all, first_above, last_above, tin_c,
                                 tout_c);
            } else {
                // the two passes below on knot pairs (same fold, same order): pass A
                double I = 0.0, eprev = 0.0, tprev = 0.0;
                for (int i = 0; i < n; i += 2) { // i <= (n−1) & ~1: the pair holds knot i
                    const double2 t2 = ld2(T, i), g2 = ld2(Gv, i), a2 = ld2(AWO, i);
                    const double e0 = sbr_exp(lam * t2.x);
                    const double ei0 = e0 * (((1.0 - g2.x) * BETA) * a2.x);
                    if (i > 0) I = I + (0.5 * (eprev + ei0)) * (t2.x - tprev);
                    eprev = ei0;
                    tprev = t2.x;
                    double e1 = 0.0;
                    if (i + 1 < n) {
                        e1 = sbr_exp(lam * t2.y);
                        const double ei1 = e1 * (((1.0 - g2.y) * BETA) * a2.y);
                        I = I + (0.5 * (eprev + ei1)) * (t2.y - tprev);
                        eprev = ei1;
                        tprev = t2.y;
                    }
                    st2(X, i, e0, e1); // X[n] (n odd) is scratch inside the capacity
                }
                const double Ieta = I;
                // pass B: HR and optimal_buffer's crossing scan (solver.jl:211-264)
                I = 0.0;
                double hr_prev = 0.0;
                for (int i = 0; i < n; i += 2) {
                    const double2 t2 = ld2(T, i), g2 = ld2(Gv, i), a2 = ld2(AWO, i), x2 = ld2(X, i);
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int k = i + h;
                        if (k >= n) break;
                        const double ti = h ? t2.y : t2.x;
                        const double xi = h ? x2.y : x2.x;
                        const double pdf = ((1.0 - (h ? g2.y : g2.x)) * BETA) * (h ? a2.y : a2.x);
                        const double ei = xi * pdf;
                        if (k > 0) I = I + (0.5 * (eprev + ei)) * (ti - tprev);
                        eprev = ei;
                        const double hr = ((p * xi) * pdf) / ((p * I) + (omp * Ieta));
                        const bool ab = hr > U;
                        any |= ab; all &= ab;
                        if (ab) { if (first_above < 0) first_above = k; last_above = k; }
                        if (k > 0) {
                            const bool abp = hr_prev > U;
                            if (!have_in && !abp && ab) {
                                tin_c = tprev + ((U - hr_prev) * (ti - tprev)) / (hr - hr_prev);
                                have_in = true;
                            }
                            if (abp && !ab) tout_c = tprev + ((U - hr_prev) * (ti - tprev)) / (hr - hr_prev);
                        }
                        hr_prev = hr;
                        tprev = ti;
                    }
                }
            }
            if (!any) { tin = ETA; tout = ETA; }
            else if (all) { tin = T[0]; tout = T[n - 1]; }
            else {
                tin = tin_c; tout = tout_c;
                if (tin == ETA) tin = T[first_above];
                if (tout == ETA) tout = T[last_above];
            }
            stamp(2);
            // ---- solve_equilibrium_baseline (solver.jl:413-462) / compute_ξ (:308-376) ----
            if (tin == tout) {
                st_r = SBR_NO_RUN_HR_BELOW_U | SBR_CONVERGED;
                tol_r = 0.0;
            } else {
                const double tolerance = 10.0 * sbr_jl_eps(a.kappa);
                double xnew = (tin + tout) / 2.0, xmin = tin, xmax = tout;
                bool boob = false;
                st_r = SBR_NO_RUN_MAXITER;
                for (int32_t k = 1; k <= a.bisect_max_iters; k++) {
                    it_r = k;
                    const double d = xmin - xmax;
                    if (collapsed(d)) { st_r = SBR_NO_RUN_COLLAPSE; break; }
                    if (k == a.bisect_max_iters - 1) { st_r = SBR_NO_RUN_MAXITER; break; }
                    const double xo = xnew;
                    const double ic = dmin(tin, xo), oc = dmin(tout, xo);
                    const double AW = interp_full(T, Gv, n, oc, boob) - interp_full(T, Gv, n, ic, boob);
                    int idx = -1;
                    if (xo >= T[0]) idx = ssl_range(T, 0, n - 1, xo);
                    if (idx < 0 || idx + 1 >= n) { st_r = SBR_OOB; break; }
                    const double eps = T[idx + 1] - T[idx];
                    const double AWe =
                        interp_full(T, Gv, n, oc + eps, boob) - interp_full(T, Gv, n, ic + eps, boob);
                    if (boob) { st_r = SBR_OOB; break; }
                    const double err = AW - a.kappa;
                    const bool inc = AWe >= AW;
                    if (fabs(err) <= tolerance) {
                        if (inc) { st_r = SBR_RUN | SBR_CONVERGED; xi_r = xo; tol_r = fabs(err); }
                        else st_r = SBR_FALSE_EQ;
                        break;
                    } else if (err > 0) {
                        xmax = xo;
                        xnew = 0.5 * (xo + xmin);
                    } else {
                        xmin = xo;
                        xnew = 0.5 * (xo + xmax);
                    }
                }
            }
        }
        stamp(3);
        if (st_r & SBR_OOB) { tin = h_oob ? (double)NAN : tin; tout = h_oob ? (double)NAN : tout; }
        if (!(st_r & SBR_RUN)) { xi_r = (double)NAN; tol_r = (st_r & SBR_NO_RUN_HR_BELOW_U) ? 0.0 : (double)INFINITY; }

        if (st_r & SBR_OOB) {
            finish = true;
            stop_oob = true;
        } else {
            bool stop = false;
            if (!(st_r & SBR_RUN)) {
                xi_n = xi_old + ETA / 500.0; // social_learning_solver.jl:150-156
                if (xi_n > ETA) stop = true;
            } else {
                xi_n = xi_r;
            }
            if (stop) {
                finish = true;
            } else {
                // get_AW(ξ_n, τ̄_IN, τ̄_OUT, HR, G_n) (solver.jl:495-532) evaluated pointwise
                const double XI = xi_n;
                const double ic = (tin >= XI) ? XI : tin;
                const double oc = (tout > XI) ? XI : tout;
                bool aoob = false;
                const double G0 = interp_full(T, Gv, n, 0.0, aoob);
                Walker wa, wb, wa2, wb2;
                wa.init(T, Gv, n); wb.init(T, Gv, n); wa2.init(T, Gv, n); wb2.init(T, Gv, n);
                auto aw_at = [&](double tau, auto& A, auto& B) {
                    const double xa = (tau - XI) + ic;
                    const double xb = (tau - XI) + oc;
                    const double gi = A.at(xa > 0 ? xa : 0.0, aoob);
                    const double go = B.at(xb > 0 ? xb : 0.0, aoob);
                    const double awin = xa >= 0 ? gi : 0.0;
                    const double awout = xb >= 0 ? go : 0.0;
                    return (awout - awin) + G0;
                };
                // ∞-norm against AW_{n-1} on range(0, η, 1000) before damping (:162-163, :195-196)
                double err = 0.0;
                {
                    Walker wt;
                    wt.init(T, T, n);
                    for (int k = 0; k < a.n_cmp; k++) {
                        const double c = CMP[k];
                        double vnew;
                        if (n < 2 || !(c >= T[0] && c <= T[n - 1])) {
                            aoob = true;
                            vnew = (double)NAN;
                        } else {
                            const int j = wt.bracket(c);
                            const double d = (c - T[j]) / (T[j + 1] - T[j]);
                            vnew = aw_at(T[j], wa, wb) * (1.0 - d) + aw_at(T[j + 1], wa2, wb2) * d;
                        }
                        const double dd = fabs(vnew - CMPO[k]);
                        if (k == 0) err = dd;
                        else if (!(err != err || err > dd)) err = dd;
                    }
                }
                stamp(4);
                if (aoob || cmp_oob) {
                    finish = true;
                    stop_oob = true;
                } else if (err < a.tol) {
                    finish = true;
                    converged = true;
                    need_awmax = (st_r & SBR_RUN) != 0;
                } else {
                    // damping α = 1/2 on G_n's knots (:174-178, :218-222): AW* at its own
                    // knot i is aw_i·(1−0) + aw_{i+1}·0 (i < n−1), aw_{n−2}·0 + aw_{n−1}·1
                    if constexpr (COOP) {
                        coop_damping(T, Gv, AWO, n, XI, ic, oc, G0, aoob);
                    } else {
                        // the same loop two knots at a time: AWO and the τ grid move in 16-byte pairs
                        WalkerV da, db;
                        da.init(T, Gv, n); db.init(T, Gv, n);
                        double2 tp = ld2(T, 0);
                        double aw_i = aw_at(tp.x, da, db);
                        for (int i = 0; i < n - 1; i += 2) {
                            // T[i+1] from the current pair, T[i+2] from the next (clamped: unused past n−1)
                            const int kn = i + 2 <= ((n - 1) & ~1) ? i + 2 : ((n - 1) & ~1);
                            const double2 tq = ld2(T, kn);
                            const double2 ao = ld2(AWO, i);
                            double aw_1 = aw_at(tp.y, da, db);
                            const double v0 = aw_i * (1.0 - 0.0) + aw_1 * 0.0;
                            const double w0 = 0.5 * ao.x + 0.5 * v0;
                            double w1;
                            if (i == n - 2) { // the pair ends the grid: AWO[n−1] takes the last segment's right end
                                const double vl = aw_i * (1.0 - 1.0) + aw_1 * 1.0;
                                w1 = 0.5 * ao.y + 0.5 * vl;
                            } else {
                                const double aw_2 = aw_at(tq.x, da, db);
                                const double v1 = aw_1 * (1.0 - 0.0) + aw_2 * 0.0;
                                w1 = 0.5 * ao.y + 0.5 * v1;
                                if (i + 1 == n - 2) {
                                    const double vl = aw_1 * (1.0 - 1.0) + aw_2 * 1.0;
                                    AWO[n - 1] = 0.5 * AWO[n - 1] + 0.5 * vl;
                                }
                                aw_1 = aw_2;
                            }
                            st2(AWO, i, w0, w1);
                            aw_i = aw_1;
                            tp = tq;
                        }
                    }
                    if (aoob) { finish = true; stop_oob = true; }
                    else if (iter >= a.max_iter) { finish = true; need_awmax = (st_r & SBR_RUN) != 0; }
                }
            }
        }
    }

    double awmax = (double)NAN;
    if (need_awmax) { // get_AW_functions!(r).AW_max (solver.jl:553-576) on r's own ξ
        const double XI = xi_r;
        const double ic = (tin >= XI) ? XI : tin;
        const double oc = (tout > XI) ? XI : tout;
        bool aoob = false;
        const double G0 = interp_full(T, Gv, n, 0.0, aoob);
        WalkerV A, B;
        A.init(T, Gv, n); B.init(T, Gv, n);
        double mx = -(double)INFINITY;
        for (int i = 0; i < n; i++) {
            const double xa = (T[i] - XI) + ic;
            const double xb = (T[i] - XI) + oc;
            const double gi = A.at(xa > 0 ? xa : 0.0, aoob);
            const double go = B.at(xb > 0 ? xb : 0.0, aoob);
            const double awin = xa >= 0 ? gi : 0.0;
            const double awout = xb >= 0 ? go : 0.0;
            const double v = (awout - awin) + G0;
            if (mx == mx && (v != v || v > mx)) mx = v;
        }
        awmax = mx;
    }

    stamp(5);
    // ---- write the iterate's SolvedModel (the oracle's `*out = r`) ----
    if (have_r) {
        a.out.xi[g] = xi_r;
        a.out.tau_in_unc[g] = tin;
        a.out.tau_out_unc[g] = tout;
        a.out.aw_max[g] = awmax;
        a.out.tol[g] = tol_r;
        a.out.status[g] = st_r;
        if (a.out.iters) a.out.iters[g] = it_r;
        if (a.path_t) { // single-point path mode (the SolvedModel's learning knots)
            if (n <= a.path_cap) {
                for (int i = 0; i < n; i++) {
                    a.path_t[i] = T[i];
                    a.path_G[i] = Gv[i];
                }
            }
            *a.path_n = n <= a.path_cap ? n : -n;
        }
    }
    if (!finish && iter >= a.max_iter) finish = true;
    if (finish) {
        uint32_t s = a.out.status[g];
        if (stop_oob) {
            a.out.xi[g] = (double)NAN;
            a.out.aw_max[g] = (double)NAN;
            a.out.tol[g] = (double)INFINITY;
            s = (s & ~(SBR_RUN | SBR_CONVERGED)) | SBR_OOB;
        }
        if (bits & SBR_KNOT_OVERFLOW) {
            a.out.xi[g] = (double)NAN;
            a.out.aw_max[g] = (double)NAN;
            a.out.tol[g] = (double)INFINITY;
            s = (s & ~(SBR_RUN | SBR_CONVERGED));
        }
        s |= bits & (SBR_ODE_MAXITERS | SBR_STIFF_SWITCH | SBR_ODE_FAILED | SBR_KNOT_OVERFLOW);
        if (!converged) s |= SBR_SOCIAL_NOT_CONVERGED;
        a.out.status[g] = s;
        if (a.fp_iters) a.fp_iters[g] = iter;
        if (a.steps_out) a.steps_out[g] = a.steps[l];
        a.live[l] = 0;
        if (a.n_live && (!COOP || (threadIdx.x & 63) == 0)) atomicSub(a.n_live, 1);
        return false;
    }
    a.live[l] = 1;
    if (a.it_cur) a.it_cur[l] = iter + 1;
    a.xi_new[l] = xi_n;
    a.n_old[l] = n;
    a.bits[l] = bits;
    // rotate: AW_n = (t_n, damped) ; free = old knots, old values, G_n
    a.slots[l] = (uint32_t)s_t | ((uint32_t)s_aw << 3) | ((uint32_t)s_to << 6) | ((uint32_t)s_vo << 9) |
                 ((uint32_t)s_G << 12);
    return true;
}

// ============================================================================
// up to n_inner fixed-point iterates for every live point of the worklist
// ============================================================================
// Lanes run their iterates back to back; the grid-wide boundary (and the
// worklist compaction after it) comes every n_inner iterates, so a launch is
// not held to the slowest point of every single iterate.
// Blocks past the main worklist's grid serve the promotion pool: slot l runs
// its own next iterates once published (a point promoted during this launch is
// picked up here or by the next launch; either way it redoes that iterate).
// args[0]: the main worklist's arguments, args[1]: the pool's (n_pts = 0: none),
// in device memory so that the wave-uniform choice between them stays scalar loads.
constexpr int kSocialWaves = 1024; // one wave per SIMD (2048 waves, two per SIMD, were slower: r04_u)
// live points up to which every point gets a whole wave (SocialRhsCoop), in rounds of the
// kSocialWaves resident ones, instead of ⌈live/kSocialWaves⌉ points per wave
constexpr int kSocialCoopMax = 4096;
// Main blocks (one wave each) spread the live worklist over all `nbs` of them: L = ⌈live/nbs⌉
// consecutive entries per wave (L ≤ 64), lanes ≥ L idle.  A fixed-point lane's RK step is a
// serial chain whose memory side grows with the wave's active lanes (each lane streams its own
// knot lines: a wave load touches one line per active lane), so as points retire the
// survivors run in ever sparser waves, down to one per wave — and with nbs = one wave per
// SIMD the bulk uses every SIMD instead of half of them.
__global__ __launch_bounds__(64, 1) void social_iter_kernel(const SocialArgs* __restrict__ args, int iter_arg,
                                                         int n_inner, const int32_t* __restrict__ work,
                                                         const int32_t* __restrict__ count, int nbs, int nmain)
{
    extern __shared__ double s_ring[]; // kRingLdsBytes: SocialRhsRing's per-lane rings
    const SocialArgs& sa = args[0];
    const SocialArgs& pa = args[1];
    const bool in_pool = (int)blockIdx.x >= nmain;
    int l, iter;
    if (!in_pool) {
        const int cnt = *count;
        // at most nmain live points: one per wave (coop), beyond that the first nbs waves
        int L = cnt <= nmain ? 1 : (cnt + nbs - 1) / nbs;
        // the ring holds kRingLanes lanes: the host's nbs = ⌈n_pts / kRingLanes⌉ >= ⌈cnt / kRingLanes⌉
        // keeps L within it; the clamp stops a future change of that arithmetic from letting lanes
        // share ring slots (which in_ring() would trust)
        constexpr int kLmax = kRingLanes;
        L = L < 1 ? 1 : (L > kLmax ? kLmax : L);
        if (L == 1) { // one point per wave: the whole wave runs it
            const int w = blockIdx.x;
            if (w >= cnt) return;
            l = work[w];
            if (!sa.live[l]) return;
            for (int k = 0; k < n_inner; k++)
                if (!social_iterate<true>(sa, l, iter_arg + k, s_ring)) break;
            return;
        }
        if ((int)threadIdx.x >= L || (int)blockIdx.x >= nbs) return;
        const int w = blockIdx.x * L + threadIdx.x;
        if (w >= cnt) return;
        l = work[w];
        if (!sa.live[l]) return; // retired by the init kernel (knot overflow)
        iter = iter_arg;
    } else {
        // one pool slot per wave, run by the whole wave (the pool holds the longest fixed
        // points — the ones whose iterates outgrew the main capacity)
        l = (int)blockIdx.x - nmain;
        if (l >= pa.n_pts) return;
        if (__hip_atomic_load(pa.ready + l, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
        if (!pa.live[l]) return;
        iter = pa.it_cur[l];
        for (int k = 0; k < n_inner; k++)
            if (!social_iterate<true>(pa, l, iter + k, s_ring)) break;
        return;
    }
    const SocialArgs& a = args[in_pool ? 1 : 0];
    for (int k = 0; k < n_inner; k++)
        if (!social_iterate<false>(a, l, iter + k, s_ring)) break;
}

// ============================================================================
// order-preserving worklist compaction: one workgroup, ballot + prefix per wave
// ============================================================================
constexpr int CMP_BLOCK = 1024;

__global__ __launch_bounds__(CMP_BLOCK) void social_compact_kernel(const int32_t* __restrict__ work_in,
                                                                   const int32_t* __restrict__ count_in,
                                                                   const int32_t* __restrict__ live,
                                                                   int32_t* __restrict__ work_out,
                                                                   int32_t* __restrict__ count_out)
{
    __shared__ int s_wave[CMP_BLOCK / 64];
    __shared__ int s_base;
    const int n = *count_in;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) s_base = 0;
    __syncthreads();
    for (int off = 0; off < n; off += CMP_BLOCK) {
        const int i = off + threadIdx.x;
        int id = 0;
        bool keep = false;
        if (i < n) {
            id = work_in[i];
            keep = live[id] != 0;
        }
        const uint64_t m = __ballot(keep);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 0) s_wave[wv] = __popcll(m);
        __syncthreads();
        int wbase = s_base;
        for (int k = 0; k < wv; k++) wbase += s_wave[k];
        if (keep) work_out[wbase + before] = id;
        __syncthreads();
        if (threadIdx.x == 0) {
            int tot = 0;
            for (int k = 0; k < CMP_BLOCK / 64; k++) tot += s_wave[k];
            s_base += tot;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) *count_out = s_base;
}

hipError_t launch_social_init(const SocialArgs& a, hipStream_t s)
{
    hipLaunchKernelGGL(social_init_kernel, dim3((a.n_pts + 63) / 64), dim3(64), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_social_iter(const SocialArgs& a, const SocialArgs& p, const SocialArgs* args_dev, int iter,
                              int n_inner, const int32_t* work, const int32_t* count, int32_t* work_out,
                              int32_t* count_out, hipStream_t s)
{
    // main blocks: one wave per SIMD of the MI355X (4 × 256), at least one wave per 64 points
    // and no more than one per point
    int nbs = (a.n_pts + kRingLanes - 1) / kRingLanes; // L = ⌈live / nbs⌉ <= kRingLanes (the ring's lanes)
    nbs = nbs > kSocialWaves ? nbs : kSocialWaves;
    nbs = nbs < a.n_pts ? nbs : (a.n_pts > 0 ? a.n_pts : 1);
    const int pool_waves = p.n_pts;
    // main blocks: nbs multi-point waves, or up to kSocialCoopMax one-point waves
    const int coop_max = kSocialCoopMax < a.n_pts ? kSocialCoopMax : a.n_pts;
    const int nmain = nbs > coop_max ? nbs : coop_max;
    hipLaunchKernelGGL(social_iter_kernel, dim3(nmain + pool_waves), dim3(64), kRingLdsBytes, s,
                       args_dev, iter, n_inner, work, count, nbs, nmain);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(social_compact_kernel, dim3(1), dim3(CMP_BLOCK), 0, s, work, count, a.live, work_out,
                       count_out);
    return hipGetLastError();
}

}  // namespace sbr
