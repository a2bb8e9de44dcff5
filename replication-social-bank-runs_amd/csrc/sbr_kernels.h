// sbr_kernels.h — argument blocks and launchers of the gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sbr {

// Per-β learning output, row-major [n_beta][cap] in HBM.
struct LearnBufs {
    double* t;          // knot times (sol.t)
    double* G;          // CDF at knots (sol.u)
    double* hr;         // hazard rate on the τ̄ grid (solver.jl:180-182)
    double* hrI;        // cumulative trapezoid ∫_0^τ̄ e^{λs} g(s) ds on the τ̄ grid
    int32_t* n_knots;   // stored knots
    int32_t* n_tau;     // length of the τ̄ grid
    int32_t* n_le;      // knots with t <= η (τ̄[i] = t[i] for i < n_le, τ̄[n_le] = η)
    uint32_t* status;   // learning-level SBR_* bits
    int32_t* n_accept;  // accepted RK steps (flop accounting)
    int32_t* n_reject;  // rejected RK steps
    int32_t cap;        // row stride (doubles) of t / G / hr / hrI: column b's row starts at b·cap
    int32_t lim;        // knots a column may store (<= cap; the learning kernel's SBR_KNOT_OVERFLOW bound)
};

struct LearnArgs {
    double x0, rtol, atol, p, lam;
    int64_t maxiters;
    int32_t n_beta;
    int32_t stop_after_eta;
    int32_t fuse_hazard; // learn_logistic_kernel: stream hazard_rate with the knots (needs hrI); 2 (the
                         // staged heads-first launch): the tail waves also normalise their rows
    // per-column readiness (single sweeps, null otherwise): the lane that finishes column b
    // takes slot k = atomicAdd(ready_tail, 1) and release-stores b + 1 into ready_q[k]
    int32_t* ready_tail;
    int32_t* ready_q;
    // hazard_kernel: the learning pdf's values on the knots (sbr_equilibrium_on_knots_pdf, e.g. the
    // social extension's (1 − G)·β·AW_{n−1}); null: compute_pdf_symbolic_baseline's βG(1 − G)
    const double* pdf = nullptr;
    // learn_logistic_kernel in one-wave blocks over grids of wpg waves each (n_beta = grids ×
    // wpg × 64, wpg > head): the first head waves of every grid take the launch's first blocks,
    // the other waves follow (0: block order = wave order)
    int32_t head = 0, wpg = 0;
    int32_t part = 0; // hazard_norm_kernel: 1 = only the head waves' columns of each grid
};

// The equilibrium side of a readiness sweep (eq_ready_kernel): one workgroup per item, each
// drawing its ticket it = atomicAdd(head, 1) < n_items when it starts; item it is tile it % tiles of the column
// published in ready_q[it / tiles] (acquire, spinning until it appears).  The tile-0 taker
// computes the column's hazard_rate and release-stores hz_flag[b] = 1; the other tiles
// acquire it before reading HR.  A wait longer than spin_limit polls gives up (status
// head[1] = 1, the tile's points unwritten): every workgroup reaches the exit.
struct ReadyArgs {
    int32_t* head;
    const int32_t* q;
    int32_t* hz_flag;
    int32_t n_items;
    int32_t tiles;
    int32_t tile_u;
    int32_t spin_limit;
};

struct EqArgs {
    double kappa;
    int32_t n_u;
    int32_t max_iters;
    int32_t lds_cap;    // knots staged in LDS per workgroup (3 doubles each + block summaries)
    double* aw_path;    // optional AW_cum(τ̄) output for single-point mode (n_u == 1)
    int32_t exhaustive; // 1: linear crossing scan + every AW knot (no block summaries)
    int32_t diag;       // SBR_FLAG_DIAG_* bits >> 8 (timing breakdown only)
    // with aw_path (baseline path mode): AW_OUT(τ̄) / AW_IN(τ̄) of get_AW (solver.jl:495-532), may be null
    double* aw_out_path;
    double* aw_in_path;
    // 1: the knots are the caller's whole interpolation grid (sbr_equilibrium_on_knots), never a
    // truncated learning solve: a lookup past the last knot is the interpolant's BoundsError
    int32_t full_grid;
    // launch_point_coop: device scratch of 3·n_tau doubles; when set, the paths are formed there and
    // copied to aw_path / aw_out_path / aw_in_path in coalesced rows (those may be mapped host memory)
    double* path_scratch;
    // compute_ξ's first iterate ξ_guess (solve_equilibrium_baseline(…; ξ_guess), solver.jl:413,441;
    // compute_ξ :309-312); NaN: the reference's default midpoint (τ̄_IN + τ̄_OUT)/2
    double xi_guess = __builtin_nan("");
    // equilibrium_kernel launched over `group` grids of gridDim.y / group columns each (the
    // pipelined batch's grouped launch): workgroups take the grids' copies of a column together
    // (dispatch index y -> column (y mod group)·per + y / group), so a heavy column's copies start
    // early instead of one per grid spread to the end of the launch
    int32_t group = 1;
};

// Interest-rate extension (sbr_baseline.hip interest mode): value function on the HR grid.
struct InterestArgs {
    double r, delta;     // interest rate, deposit maturity rate (0 ≤ r < δ); r = 0: the baseline
    double rtol, atol;   // value-function Tsit5 tolerances (value_function_solver.jl:66: eps())
    int64_t maxiters;
    int64_t* steps;      // value-function RK steps per point (may be null)
    double* v_path;      // single-point mode (n_u = 1): V on the HR grid (may be null)
    int32_t* v_count;    // ... and the number of saved values
};

struct ResultSoA {
    double *xi, *tau_in_unc, *tau_out_unc, *aw_max, *tol;
    uint32_t* status;
    int32_t* iters;
};

// Hetero learning output: t [n_col][cap], G [n_col][cap][K], hr/hrI [n_col][K][cap].
struct HeteroBufs {
    double* t;
    double* G;
    double* hr;
    double* hrI;
    int32_t* n_knots;
    int32_t* n_tau;
    int32_t* n_le;
    uint32_t* status;
    int32_t* n_accept;
    int32_t* n_reject;
    int32_t cap; // row stride (knots) of t, G and the K hazard rows
    int32_t lim; // knots a column may store (<= cap; SBR_KNOT_OVERFLOW beyond)
};

struct HeteroEqArgs {
    double kappa;
    double tolerance;   // compute_ξ_hetero tolerance (1e-12 absolute)
    int32_t n_u;
    int32_t max_iters;  // 500
    int32_t lds_cap;    // knot times staged in LDS
    int32_t exhaustive; // 1: evaluate AW over every knot (no branch and bound)
    int32_t diag;       // SBR_FLAG_DIAG_* bits >> 8 (timing breakdown only)
    double* aw_path;    // single-point mode (n_u = 1): AW_total on the learning knots (may be null)
    int32_t n_col;      // set by the launcher (XCD-aware 1-D grid)
};

// Promotion pool of the social sweep: a point whose iterate outgrows the knot
// capacity moves (AW_{n-1} and its carried state) into a free slot here and
// redoes that iterate from the pool blocks of the same or the next launch,
// concurrently with the main worklist.
struct SocialPool {
    double* ws;          // [n_slots][5][cap] wave-blocked like the main workspace
    int32_t cap;
    int32_t n_slots;
    int32_t* used;       // slot allocator (atomic counter)
    int32_t* n_live;     // promoted points not finished yet
    int64_t* pts;        // slot -> global point
    int32_t* n_old;
    uint32_t* slots;
    double* xi_new;
    uint32_t* bits;
    int64_t* steps;
    int32_t* live;
    int32_t* it_cur;     // next iterate of the slot's point
    int32_t* ready;      // 1 once the slot's state is published (release / acquire)
};

// Social-learning fixed point (sbr_social.hip): one lane per point; per-point
// workspace of 5 knot buffers × cap doubles (wave-blocked) + n_cmp doubles.
struct SocialArgs {
    const double* beta;  // [n_beta]
    const double* eta;   // [n_beta]
    const double* u;     // [n_u]
    const double* cmp;   // [n_beta][n_cmp] comparison grids range(0, η, n_cmp)
    int64_t pt0;         // first global point (β-major, u-fastest) of this chunk
    const int64_t* pts;  // or: explicit global point indices (overflow retries), may be null
    int32_t n_pts;       // points in this chunk
    int32_t n_u;
    int32_t n_cmp;
    int32_t max_iter;    // fixed-point iterations (script: 500)
    int32_t bisect_max_iters;
    int32_t cap;         // knots per buffer
    int64_t maxiters;    // ODE maxiters
    double x0, p, kappa, lam, tol, rtol, atol;
    double* ws;          // [n_pts][5][cap]
    double* cmpo;        // [n_pts][n_cmp]
    int32_t* n_old;      // knots of AW_{n-1}
    uint32_t* slots;     // buffer permutation (5 × 3 bits)
    double* xi_new;      // ξ carried between iterates
    uint32_t* bits;      // accumulated ODE status bits
    int64_t* steps;      // RK steps attempted (accepted + rejected), all iterates
    int32_t* live;       // 1 while the point iterates
    int32_t* work;       // initial worklist (filled by the init kernel)
    int32_t* count;      // initial worklist length
    ResultSoA out;       // global result arrays (indexed pt0 + local)
    int32_t* fp_iters;   // fixed-point iterations (may be null)
    int64_t* steps_out;  // RK steps per point, written when it finishes (may be null)
    int64_t* prof;       // diagnostics [n_pts][8] cycles per phase + counters (may be null)
    SocialPool pool;     // large-capacity slots for points that outgrow `cap` (ws null: none)
    // set on the pool's own arguments only: per-point iterate, published flag, live counter
    int32_t* it_cur;
    int32_t* ready;
    int32_t* n_live;
    // single-point path mode: the learning knots of every iterate's equilibrium (the
    // returned SolvedModel's are the last written); path_n = knots (−knots if > path_cap)
    double* path_t;
    double* path_G;
    double* path_aw;     // AW_{n-1} at the knots (the forcing of compute_pdf_social_learning), may be null
    int32_t* path_n;
    int32_t path_cap;
};

hipError_t launch_social_init(const SocialArgs& a, hipStream_t s);
// n_inner iterates (from `iter`) over `work`/`count` plus every published pool
// slot (`p`, n_pts = 0: no pool), then the ordered compaction of the main
// worklist into work_out; args_dev holds {a, p} in device memory
hipError_t launch_social_iter(const SocialArgs& a, const SocialArgs& p, const SocialArgs* args_dev, int iter,
                              int n_inner, const int32_t* work, const int32_t* count, int32_t* work_out,
                              int32_t* count_out, hipStream_t s);

// phase 0: learning (+ the streamed hazards); 1: equilibria; 2: the hazards of knots and group
// CDFs already in L (n_knots and status set by the caller)
// get_AW_hetero's per-group AW_OUT_k / AW_IN_k on one solved point's knots (T [n], G [n][K],
// n = *n_dev <= n_max; ξ, τ̄_IN [K], τ̄_OUT [K], status on the device): rows of stride ld
hipError_t launch_hetero_aw_groups(int K, const double* T, const double* G, const int32_t* n_dev, int n_max,
                                   const double* xi, const double* tin, const double* tout, const uint32_t* status,
                                   double* out, size_t ld, hipStream_t s);
hipError_t launch_hetero(int K, const double* betas, const double* dist, const double* eta, const double* t_end,
                         const double* u, const LearnArgs& la, const HeteroEqArgs& ea, const HeteroBufs& L,
                         const ResultSoA& out, double* tin, double* tout, hipStream_t s, int phase);

hipError_t launch_learn_logistic(const double* beta, const double* eta, const double* t_end, const LearnArgs& a,
                                 const LearnBufs& L, hipStream_t s);
// the learning kernel alone (a.fuse_hazard: HR numerators and running integrals streamed, to be
// normalised by launch_hazard_norm); mode 0: two waves per workgroup (beside a running equilibrium
// launch), 1: one wave per workgroup (latency), 2: a batch's wide learning launch (the chip otherwise idle:
// LDS-staged rows; a.fuse_hazard must be 1, launch_hazard_norm follows)
hipError_t launch_learn_kernel(const double* beta, const double* eta, const double* t_end, const LearnArgs& a,
                               const LearnBufs& L, hipStream_t s, int mode);
// HR = numerator / (p·I + (1 − p)·I_η) over the first n_cols columns of L (after a fused learning)
hipError_t launch_hazard_norm(const LearnArgs& a, const LearnBufs& L, int n_cols, hipStream_t s);
// only_mode: 0 = the LDS-slab launch then the global-memory launch; 1 / 2 = only one of them
// (a caller that knows every column fits the slab, or none does).  a.aw_path (n_u == 1): the
// solving lane writes AW_cum on τ̄ (exhaustive); single points use launch_point_coop instead.
hipError_t launch_equilibrium(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                              const EqArgs& a, const ResultSoA& out, int n_beta, hipStream_t s, int only_mode = 0);
// one point per workgroup (u[j], results at [j], j < n_points; column 0 of L): wave-wide searches for the solve,
// the block for get_AW's exhaustive pass (AW_max and, with a.aw_path, the three paths).  a.lds_cap
// = knots staged per array (3 arrays: t, G, HR); larger columns run from global memory.
hipError_t launch_point_coop(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                             const EqArgs& a, const ResultSoA& out, hipStream_t s, int n_points = 1);
// hazard_rate (solver.jl:153-185) of n_beta columns whose knots, n_knots, n_le (#knots <= η) and
// status are in L (the hazard stage of launch_learn_logistic on its own)
hipError_t launch_hazard(const double* beta, const double* eta, const LearnArgs& a, const LearnBufs& L, int n_beta,
                         hipStream_t s);
// the equilibrium side of a readiness sweep: one workgroup per item (hazard + equilibria
// of each column as soon as the learning kernel publishes it); the learning side is
// launch_learn_logistic with la.ready_q set and la.fuse_hazard = 0, without its hazard launch
hipError_t launch_eq_ready(const LearnBufs& L, const double* beta, const double* eta, const double* t_end,
                           const double* u, const LearnArgs& la, const EqArgs& a, const ReadyArgs& ra,
                           const ResultSoA& out, int n_blocks, hipStream_t s);
// after a readiness sweep, on the stream that orders after it: if a workgroup gave up waiting
// (*gave_up != 0), every one of the n_pts points is marked SBR_ENGINE_SCHED (ξ = AW_max = NaN,
// tol = Inf) — the failure is visible in the results without a host synchronisation
hipError_t launch_ready_fail(const int32_t* gave_up, const ResultSoA& out, int64_t n_pts, hipStream_t s);
// solve_equilibrium_interest per (β, u) on the same learning buffers
hipError_t launch_interest(const LearnBufs& L, const double* eta, const double* t_end, const double* u,
                           const EqArgs& a, const InterestArgs& ia, const ResultSoA& out, int n_beta, hipStream_t s);

}  // namespace sbr
