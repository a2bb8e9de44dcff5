/*
 * sbr.h — C ABI of libsbr, the MI355X batched equilibrium engine for
 * "The Social Determinants of Bank Runs" (Robin-Lenoir/replication-social-bank-runs).
 *
 * The reference has no FFI: its "interface" is a set of Julia functions that
 * the scripts call point by point.  Each entry point below
 * replaces one of those call patterns with a batched call; a Julia caller
 * binds them with `ccall` (see INTEGRATION.md for the shim).
 *
 * Conventions
 *  - plain C types only; every array is caller-allocated;
 *  - result arrays are n_beta*n_u long, u-fastest: element (i, j) — the i-th β
 *    and the j-th u — is at [i*n_u + j]; this is max_AW_matrix[j, i] of
 *    scripts/1_baseline.jl:213,254;
 *  - functions return 0 on success or a negative SBR_E* code;
 *  - per-point outcomes are status bits (sbr_status.h); xi is NaN and tol is
 *    Inf whenever SBR_RUN is clear, exactly like SolvedModel
 *    (src/baseline/solver.jl:429-455);
 *  - a context is bound to one HIP device; calls on one context are
 *    serialised by the caller; distinct contexts are independent.
 *  - The *_dev variants take device pointers and a hipStream_t (as void*) and
 *    do not synchronise: they are what the multi-GPU host layer and the
 *    benchmark use (inputs already resident in HBM).
 */
#ifndef SBR_H
#define SBR_H

#include <stdint.h>

#include "sbr_status.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SBR_OK 0
#define SBR_EARG (-1)    /* ArgumentError of model.jl:31-35,71-76 / heterogeneity_model.jl:33-41 */
#define SBR_EDEVICE (-2) /* HIP runtime error or no device */
#define SBR_ENOMEM (-3)  /* device allocation failed */

typedef struct sbr_ctx sbr_ctx;

typedef struct {
    double ode_reltol;          /* learning.jl:43 reltol = eps() (0 = eps(): every zero field is the default) */
    double ode_abstol;          /* learning.jl:43 abstol = eps() (0 = eps()) */
    int64_t ode_maxiters;       /* OrdinaryDiffEq default maxiters = 1e6 (SBR_DEFAULT_ODE_MAXITERS) */
    int32_t bisect_max_iters;   /* solver.jl:309 max_iters = 100 */
    int32_t early_exit_nan_run; /* 1_baseline.jl:147,221: 5; 0 disables */
    int32_t knot_capacity;      /* engine limit on stored knots per β (0 = default 65536) */
    int32_t hetero_max_iters;   /* heterogeneity_solver.jl:49 max_iters = 500 */
    int32_t flags;              /* SBR_FLAG_* */
    int32_t pad;                /* social sweep: knot capacity per buffer (0 = default 98304) */
    double xi_guess;            /* solver.jl:413,441 ξ_guess: compute_ξ's first iterate, read only with
                                   SBR_FLAG_XI_GUESS (a zero-filled opts is the default midpoint
                                   (τ̄_IN + τ̄_OUT)/2).  sbr_equilibrium_on_knots[_pdf] only: the other
                                   entry points return SBR_EARG when the flag is set */
} sbr_opts;

/* Evaluate every τ̄ knot of the crossing scan and of the AW path (no block
 * summaries / branch-and-bound).  Same results; for A/B timing and checks. */
#define SBR_FLAG_EXHAUSTIVE 0x1
/* Single sweeps (sbr_sweep_baseline[_dev]): per-column readiness instead of the default
 * three-chunk schedule — the learning kernel publishes each column the moment its lane has
 * solved it, and one equilibrium workgroup per column (on CUs the learning waves do not
 * use) runs its hazard and equilibria.  Same results; slower on the configs (the columns'
 * learning ends late and the equilibria lose the learning CUs), kept for A/B. */
#define SBR_FLAG_READY_SWEEP 0x2 /* a timed-out wait marks every point SBR_ENGINE_SCHED (_dev) / SBR_EDEVICE (host) */
/* n-device contexts (sbr_init_multi): return the host-pointer sweep's results through an RCCL
 * gather of every rank's block to device 0 over xGMI and one scatter from there, instead of
 * the default direct transport (each GPU copies its own columns into the caller's arrays over
 * its own PCIe link, no collective).  Same results. */
#define SBR_FLAG_RCCL_GATHER 0x4
/* opts->xi_guess holds compute_ξ's first iterate (solve_equilibrium_baseline(...; ξ_guess),
 * solver.jl:413,441); without this flag xi_guess is ignored and the midpoint is used. */
#define SBR_FLAG_XI_GUESS 0x8
/* Diagnostics (timing breakdown only — results are NOT the reference's):
 * stop every point after the crossing scan / after the ξ bisection, or
 * report the number of 64-knot AW blocks evaluated in `iters` instead of
 * the bisection count.  In the hetero sweep 0x400 stops after the validity
 * check instead. */
#define SBR_FLAG_DIAG_STOP_AFTER_BUFFER 0x100
#define SBR_FLAG_DIAG_STOP_AFTER_BISECT 0x200
#define SBR_FLAG_DIAG_COUNT_AW_BLOCKS 0x400
/* Diagnostics of the social sweep: per-phase shader-cycle sums, read with
 * sbr_social_prof_read (results unchanged). */
#define SBR_FLAG_DIAG_SOCIAL_PROF 0x800

typedef struct {
    double* xi;          /* SolvedModel.ξ                       */
    double* tau_in_unc;  /* SolvedModel.τ_bar_IN_UNC            */
    double* tau_out_unc; /* SolvedModel.τ_bar_OUT_UNC           */
    double* aw_max;      /* get_AW_functions!(...).AW_max       */
    double* tol;         /* SolvedModel.tolerance               */
    uint32_t* status;    /* SBR_* bits                          */
    int32_t* iters;      /* bisection iterations (may be NULL)  */
} sbr_result_soa;

/* Fills *o with the reference defaults (eps() tolerances, 1e6, 100, 5, 65536, 500, no ξ_guess). */
void sbr_default_opts(sbr_opts* o);

/* Creates a context on HIP device `device` (the caller's rank-local GPU). */
int sbr_init(int device, sbr_ctx** ctx);
int sbr_free(sbr_ctx* ctx);
const char* sbr_last_error(const sbr_ctx* ctx);

/*
 * n-device context (SURVEY.md §8(b) `sbr_init(n_gpus, …)`, §8(e)): n_gpus HIP devices
 * (`devices` lists their ids, NULL = 0 .. n_gpus-1), one single-device context per device.
 * The host-pointer sweeps — sbr_sweep_baseline, sbr_sweep_hetero, sbr_sweep_social,
 * sbr_sweep_interest — on such a context deal the parameter columns cyclically (column i
 * to device i mod n_gpus) and solve every shard on its GPU from one host thread per GPU.
 * Results travel by the direct transport (default): each GPU copies its own packed result
 * block in one DMA over its own PCIe link into a pinned landing buffer, and once every rank
 * has succeeded host threads copy the columns into the caller's arrays — no collective runs,
 * nothing funnels through device 0, and a failed call writes none of the caller's arrays.
 * With SBR_FLAG_RCCL_GATHER the blocks are gathered to device 0 over RCCL (xGMI) and
 * scattered from there instead; librccl.so.1 is loaded and the communicators created only
 * then (that transport is unverified on multi-GPU hardware).  Either way the results are in
 * the single-device layout, bit-identical to a one-GPU sweep (per-point results do not
 * depend on the partitioning).  Single-point, learning-only and diagnostic calls run on
 * device 0; the device-pointer (*_dev) entry points need a single-device context:
 * sbr_multi_child(ctx, rank).  A call is synchronous; contexts are independent, so
 * distinct contexts may be used from distinct threads.  Diagnostic: with the environment
 * variable SBR_MULTI_SHARED_DEVICES=1, ranks may share a device (duplicate ids, or rank r
 * on device r mod count) — the n-rank fan-out rehearsed on fewer GPUs; the RCCL gather is
 * refused (SBR_EARG) on such a context.
 */
int sbr_init_multi(int n_gpus, const int* devices, sbr_ctx** ctx);
/* number of devices of a context (1 for sbr_init's) */
int sbr_multi_size(const sbr_ctx* ctx);
/* the single-device context of rank `rank` (rank 0 of a single-device context is itself) */
sbr_ctx* sbr_multi_child(sbr_ctx* ctx, int rank);

/*
 * Baseline β×u sweep — replaces the Fig 4/Fig 5 loops of
 * scripts/1_baseline.jl:151-192 and :224-267, i.e. for each β
 *     lr = solve_learning(LearningParameters(β, (0, t_end[i]), x0))   learning.jl:109
 * and for each u
 *     r  = solve_equilibrium_baseline(lr, EconomicParameters(u, p, κ, λ, η_bar, η[i]))  solver.jl:413
 *     get_AW_functions!(r).AW_max                                         solver.jl:553-576
 * eta/t_end are per-β so that the copy-modify carry-over of model.jl:189-211
 * (η = 15, tspan = (0, 30) for every β of Fig 5) is expressed by the caller.
 * Host pointers; synchronous.
 */
int sbr_sweep_baseline(sbr_ctx* ctx, const double* beta, const double* eta, const double* t_end, double x0,
                       const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                       const sbr_opts* opts, sbr_result_soa* out);

/* Same on device pointers (beta/eta/t_end/u and every out field in HBM),
 * enqueued on `stream` (hipStream_t; NULL is HIP's null stream, i.e. torch's default
 * stream, never a private one); no host synchronisation. */
int sbr_sweep_baseline_dev(sbr_ctx* ctx, void* stream, const double* beta, const double* eta,
                           const double* t_end, double x0, const double* u, int64_t n_beta, int64_t n_u, double p,
                           double kappa, double lambda, const sbr_opts* opts, sbr_result_soa* out);

/*
 * n_batch grids that share n_beta, n_u, u and the scalars (the Fig 5 loop of
 * scripts/1_baseline.jl:224-267 for n_batch parameter grids), swept back to back.
 * The learning stage is latency-bound (one serial ODE per β lane), so the grids
 * are learned together — as many as fit one learning launch of at most one wave
 * per SIMD and the workspace budget (sbr_set_batch_workspace) — and their
 * equilibria then run back to back; a longer batch learns its next group into a
 * second workspace beside those equilibria.  beta/eta/t_end are
 * [n_batch × n_beta] (row k = batch k); every out field is
 * [n_batch × n_beta × n_u] (iters may be NULL).  Device pointers; inputs are read
 * after the work already enqueued on `stream`, results are complete for work
 * enqueued on `stream` afterwards.  Each batch gives exactly what
 * sbr_sweep_baseline_dev gives for it.  Use a context from one stream at a time.
 */
int sbr_sweep_baseline_batch_dev(sbr_ctx* ctx, void* stream, int64_t n_batch, const double* beta,
                                 const double* eta, const double* t_end, double x0, const double* u,
                                 int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                                 const sbr_opts* opts, sbr_result_soa* out);
/* Size (allocate) now the workspaces a later sbr_sweep_baseline_batch_dev of n_batch grids of
 * n_beta columns with these opts (knot_capacity) will use, so that the call itself allocates
 * nothing — the HBM allocator's work stays out of a timed loop.  Waits for the context's
 * earlier work.  The batch call re-sizes by itself when needed; this is never required. */
int sbr_batch_reserve(sbr_ctx* ctx, int64_t n_batch, int64_t n_beta, const sbr_opts* opts);
/* Budget in bytes for the learning workspaces of baseline batches (0 = 40 % of the free plus
 * already held HBM at call time): it caps the grids learned per launch (each grid takes
 * n_beta × (4 × knot_capacity × 8 + 24) bytes, two workspaces when the batch needs more than
 * one group).  An allocation that fails anyway halves the group and retries, down to one grid. */
int sbr_set_batch_workspace(sbr_ctx* ctx, int64_t bytes);

/*
 * Make `stream` wait (device side, no host sync) until grid k of the last
 * sbr_sweep_baseline_batch_dev call on this context has its results, while the
 * later grids of the batch are still being swept: the caller can ship grid k's
 * results (e.g. an RCCL gather to rank 0, the collection of the result matrix
 * in scripts/1_baseline.jl:224-267) overlapped with the rest of the batch.
 * SBR_EARG if k is not a grid of that call.
 */
int sbr_batch_wait(sbr_ctx* ctx, void* stream, int64_t k);

/*
 * Learning only — solve_learning (learning.jl:109-124) for n_beta β at once.
 * Writes, per β, the knot grid t and CDF values G of the adaptive ODE
 * solution (row i at [i*cap .. i*cap + n_knots[i]) ); g = βG(1−G) is implied
 * (learning.jl:161-173).  When stop_after_eta != 0 the integration stops at
 * the first knot the equilibrium stage can never read, else
 * it runs to t_end like the reference.  Host pointers; synchronous.
 */
int sbr_learn_baseline(sbr_ctx* ctx, const double* beta, const double* eta, const double* t_end, double x0,
                       int64_t n_beta, int32_t stop_after_eta, const sbr_opts* opts, double* t_out, double* G_out,
                       int64_t cap, int32_t* n_knots, uint32_t* status);

/*
 * Single point with paths — solve_learning + solve_equilibrium_baseline +
 * get_AW (solver.jl:495-532) for one (β, u), returning the hazard grid τ̄,
 * HR(τ̄) and AW_cum(τ̄) (arrays of length *n_tau, capacity cap) so that a
 * caller can rebuild the LinearInterpolation objects the reference's
 * plotting code consumes.  res = {ξ, τ̄_IN, τ̄_OUT, AW_max, tol}.
 */
int sbr_solve_point_paths(sbr_ctx* ctx, double beta, double eta, double t_end, double x0, double u, double p,
                          double kappa, double lambda, const sbr_opts* opts, double* res, uint32_t* status,
                          double* tau, double* hr, double* aw_cum, int64_t cap, int64_t* n_tau);

/*
 * Equilibria on the caller's learning knots — for one LearningResults `lr` and n_u values of u
 * sharing (p, κ, λ, η):
 *     r = solve_equilibrium_baseline(lr, EconomicParameters(u_j, p, κ, λ, η_bar, η))  solver.jl:413-462
 *     get_AW_functions!(r)                                                        solver.jl:553-576
 * with lr's own knot grid — t, G = the knots and values of lr.learning_cdf (learning.jl:52),
 * beta = lr.params.β for the symbolic pdf βG(1−G) (learning.jl:161-173), t_end =
 * lr.params.tspan[2] (optimal_buffer's no-crossing value, solver.jl:221-223, 424) — and no
 * learning ODE: the scripts learn once per β and call this per u (1_baseline.jl:44 / :169,
 * :227 / :248).  The knots and the u-independent hazard path stay resident on the device: a
 * call whose t, G (compared by value), β, η, p and λ equal the previous call's uploads only u.
 * Lookups outside [t[0], t[n−1]] are the interpolant's BoundsError (SBR_OOB); t must be sorted
 * (SBR_EARG otherwise, like Interpolations).  Results: n_u entries per out field (host).
 * Paths (each may be NULL; capacity cap): tau / hr = the hazard grid τ̄ and HR(τ̄) (*n_tau
 * entries, 0 after the hazard's BoundsError); with n_u == 1, aw_cum / aw_out / aw_in =
 * AW_cum, AW_OUT, AW_IN on τ̄ (get_AW, solver.jl:495-532; NaN without a run).  Synchronous.
 */
int sbr_equilibrium_on_knots(sbr_ctx* ctx, const double* t, const double* G, int64_t n_knots, double beta,
                             double eta, double t_end, const double* u, int64_t n_u, double p, double kappa,
                             double lambda, const sbr_opts* opts, sbr_result_soa* out, double* tau, double* hr,
                             double* aw_cum, double* aw_out, double* aw_in, int64_t cap, int64_t* n_tau);

/*
 * The same on an explicit learning pdf: pdf[i] = the pdf's value at knot t[i] (n_knots values;
 * its LinearInterpolation feeds hazard_rate(p, λ, pdf, η), solver.jl:153-185) instead of
 * βG(1−G).  The social drop-in's final SolvedModel (social_learning_solver.jl:139-143, 262) is
 * this call on the last iterate's knots with pdf = (1 − G)·β·AW_{n−1}
 * (compute_pdf_social_learning, social_learning_dynamics.jl:98-114): its HR and AW paths are
 * the social point's, bit for bit.  Residency is keyed by t, G, pdf, η, p, λ.
 */
int sbr_equilibrium_on_knots_pdf(sbr_ctx* ctx, const double* t, const double* G, const double* pdf,
                                 int64_t n_knots, double eta, double t_end, const double* u, int64_t n_u, double p,
                                 double kappa, double lambda, const sbr_opts* opts, sbr_result_soa* out, double* tau,
                                 double* hr, double* aw_cum, double* aw_out, double* aw_in, int64_t cap,
                                 int64_t* n_tau);

/*
 * Heterogeneity extension sweep — for each column c (group rates
 * betas[c*K .. c*K+K), η = eta[c], tspan = (0, t_end[c])):
 *     lr = solve_SInetwork_hetero(LearningParametersHetero(βs, dist, tspan, x0))  heterogeneity_learning.jl:49
 * and for each u:
 *     r  = solve_equilibrium_hetero(lr, EconomicParameters(u, p, κ, λ, η_bar, η))  heterogeneity_solver.jl:241
 *     get_AW_functions_hetero!(r).AW_max                                            heterogeneity_solver.jl:386
 * K ∈ {1, 2, 3, 4, 8}.  out->tau_in_unc/tau_out_unc are ignored; the per-group
 * buffers go to tau_in/tau_out ([n_col*n_u][K], may be NULL).  The caller
 * resolves η = η_bar / Σ dist·βs per column (heterogeneity_model.jl:131-132).
 */
/*
 * Heterogeneity learning only — solve_SInetwork_hetero (heterogeneity_learning.jl:49-94) for
 * n_col columns at once (column c: group rates betas[c*K .. c*K+K), tspan = (0, t_end[c])):
 * the shared knot grid t (row c at [c*cap ..]) and the group CDFs G (row c at [c*cap*K ..],
 * knot-major: G[c][i][k]) of the AutoTsit5(Rosenbrock23()) solution at eps() tolerance, run to
 * t_end like the reference; the PDFs follow from compute_pdf_hetero (:114-134).  Validation
 * mirrors LearningParametersHetero (heterogeneity_model.jl:33-41).  Host pointers; synchronous.
 */
int sbr_learn_hetero(sbr_ctx* ctx, int32_t K, const double* betas, const double* dist, const double* t_end, double x0,
                     int64_t n_col, const sbr_opts* opts, double* t_out, double* G_out, int64_t cap, int32_t* n_knots,
                     uint32_t* status);

int sbr_sweep_hetero(sbr_ctx* ctx, int32_t K, const double* betas, const double* dist, const double* eta,
                     const double* t_end, double x0, const double* u, int64_t n_col, int64_t n_u, double p,
                     double kappa, double lambda, const sbr_opts* opts, sbr_result_soa* out, double* tau_in,
                     double* tau_out);
int sbr_sweep_hetero_dev(sbr_ctx* ctx, void* stream, int32_t K, const double* betas, const double* dist,
                         const double* eta, const double* t_end, double x0, const double* u, int64_t n_col,
                         int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
                         sbr_result_soa* out, double* tau_in, double* tau_out);

/*
 * n_batch heterogeneity grids that share K, dist, n_col, n_u, u and the scalars, swept back
 * to back and pipelined like sbr_sweep_baseline_batch_dev: the learning of batch k+1
 * (solve_SInetwork_hetero, latency-bound: one lane per column) runs on a highest-priority
 * stream into the second of two workspaces while the equilibrium of batch k fills the CUs.
 * betas is [n_batch × n_col × K], eta/t_end [n_batch × n_col], every out field
 * [n_batch × n_col × n_u] (iters may be NULL), tau_in/tau_out [n_batch × n_col × n_u × K]
 * or NULL.  Device pointers, enqueued on `stream`; each batch gives exactly what
 * sbr_sweep_hetero_dev gives for it.  Use a context from one stream at a time.
 */
int sbr_sweep_hetero_batch_dev(sbr_ctx* ctx, void* stream, int64_t n_batch, int32_t K, const double* betas,
                               const double* dist, const double* eta, const double* t_end, double x0,
                               const double* u, int64_t n_col, int64_t n_u, double p, double kappa, double lambda,
                               const sbr_opts* opts, sbr_result_soa* out, double* tau_in, double* tau_out);
/*
 * Heterogeneity equilibria on the caller's learning knots — solve_equilibrium_hetero(lr_hetero,
 * econ) + get_AW_functions_hetero! (heterogeneity_solver.jl:241-293, 316-402) for one
 * LearningResultsHetero: its knot grid t[n] and group CDF values G[n][K] (knot-major, the
 * learning_cdfs' coefficients, heterogeneity_learning.jl:82-86), its βs / dist (learning.params;
 * the pdfs follow from compute_pdf_hetero, :114-134) and tspan end t_end; n_u values of u sharing
 * (p, κ, λ, η).  No learning ODE runs: the scripts learn once (2_heterogeneity.jl:59) and solve per
 * u.  Knots, group CDFs and the K hazard paths stay resident while the inputs repeat (compared by
 * value), like sbr_equilibrium_on_knots.  out->tau_in_unc / tau_out_unc are ignored; the per-group
 * buffers go to tau_in / tau_out ([n_u][K], may be NULL).  Paths (may be NULL, capacity cap):
 * hr = HR_k on the τ̄ grid (knots <= η, then η: hazard_rate's explicit grid, solver.jl:163-164) at
 * hr + k·cap, *n_tau entries each (0 after the hazard's BoundsError) — SolvedModelHetero.HRs
 * (:255); with n_u == 1, aw_total = AW_total on the knots and aw_groups = get_AW_hetero's per-group
 * curves on the knots (:335-362): AW_OUT_k at aw_groups + k·cap, AW_IN_k at aw_groups + (K + k)·cap
 * (each may be NULL; NaN rows without a run, where get_AW_hetero returns nothing).  Synchronous.
 */
int sbr_hetero_equilibrium_on_knots(sbr_ctx* ctx, int32_t K, const double* t, const double* G, int64_t n_knots,
                                    const double* betas, const double* dist, double eta, double t_end, const double* u,
                                    int64_t n_u, double p, double kappa, double lambda, const sbr_opts* opts,
                                    sbr_result_soa* out, double* tau_in, double* tau_out, double* hr, double* aw_total,
                                    double* aw_groups, int64_t cap, int64_t* n_tau);

/* One heterogeneity equilibrium with what scripts/2_heterogeneity.jl plots
 * (aggregate_withdrawals_hetero.pdf): learning knots t[n] and group CDFs G[n][K]
 * (solve_SInetwork_hetero), the per-group buffers, and AW_total on the knots
 * (get_AW_functions_hetero!, heterogeneity_solver.jl:386; NaN without a run) and each
 * group's curves AW_OUT_k / AW_IN_k on the knots (get_AW_hetero, :335-362; aw_groups rows
 * k and K + k, stride cap).  res = {ξ, AW_max, tol}; t / aw_total hold `cap` doubles,
 * G cap·K, aw_groups 2K·cap (any of them may be NULL). */
int sbr_hetero_point_paths(sbr_ctx* ctx, int32_t K, const double* betas, const double* dist, double eta, double t_end,
                           double x0, double u, double p, double kappa, double lambda, const sbr_opts* opts,
                           double* res, uint32_t* status, double* tau_in, double* tau_out, double* t, double* G,
                           double* aw_total, double* aw_groups, int64_t cap, int64_t* n_knots);

/*
 * Social-learning extension sweep — for each β column b and each u:
 *     solve_equilibrium_social_learning(ModelParameters(β_b, η_b, u, p, κ, λ, x0); tol, max_iter)
 *                                          social_learning_solver.jl:63-263
 *     get_AW_functions!(result).AW_max     solver.jl:553-576
 * i.e. the fixed point between learning from aggregate withdrawals
 * (social_learning_dynamics.jl:58-114) and the baseline equilibrium, damped
 * by 1/2, with tspan = (0, η) (:79).  cmp_grid is [n_beta × n_cmp]: row b is
 * collect(range(0.0, η_b, length = 1000)) of :103 (passed in so that a Julia
 * caller hands over Julia's own range elements).  Results are the returned
 * SolvedModel (the last inner equilibrium, :262) u-fastest; the fixed-point
 * outcome is SBR_SOCIAL_NOT_CONVERGED (max_iter reached, ξ search past η, or a
 * BoundsError of the reference: SBR_OOB) and fp_iters (may be NULL);
 * rk_steps (may be NULL) = Tsit5 steps attempted per point, for flop counts.
 * Host pointers; synchronous.  The HBM workspace is 5 × capacity doubles per
 * point in flight (opts->pad, default 98304 knots: ≈3.9 MB); large grids run
 * in chunks that fit sbr_set_social_workspace (default 60 % of free HBM).
 * A point whose iterate outgrows the capacity (the non-converging fringe of
 * config 5 reaches 450k knots) moves with its AW_{n-1} into a pool of up to
 * 256 slots of 16× the capacity (held beside the workspace, ≤ 15 % of free
 * HBM) and redoes that iterate there within the same sweep; a point that
 * outgrows the pool too, or finds it full, is re-run from scratch at 4× the
 * pool capacity, up to 4M knots, so results equal an unbounded grid's; only
 * beyond that does a point end with SBR_KNOT_OVERFLOW.
 */
int sbr_sweep_social(sbr_ctx* ctx, const double* beta, const double* eta, double x0, const double* u, int64_t n_beta,
                     int64_t n_u, double p, double kappa, double lambda, const double* cmp_grid, int32_t n_cmp,
                     double tol, int32_t max_iter, const sbr_opts* opts, sbr_result_soa* out, int32_t* fp_iters,
                     int64_t* rk_steps);
/* Same on device pointers, enqueued on `stream` (all max_iter iterates are
 * launched; finished points drop out of the worklist).  The stream is
 * synchronised once at the end to find knot-capacity overflows (re-run as
 * above); the call returns when every point is final. */
int sbr_sweep_social_dev(sbr_ctx* ctx, void* stream, const double* beta, const double* eta, double x0,
                         const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda,
                         const double* cmp_grid, int32_t n_cmp, double tol, int32_t max_iter, const sbr_opts* opts,
                         sbr_result_soa* out, int32_t* fp_iters, int64_t* rk_steps);
/* One social-learning fixed point with the learning knots t[n], G[n] of the
 * returned SolvedModel (the last inner equilibrium, social_learning_solver.jl:262)
 * — with ξ, τ̄_IN, τ̄_OUT they rebuild the AW curves scripts/4_social_learning.jl
 * plots (get_AW on τ̄ = knots ≤ η (+ η)).  aw_old (may be NULL) receives
 * AW_{n-1}(t_i), the forcing that drove that iterate, so that the caller rebuilds
 * its learning_pdf = (1 − G)·β·AW_{n-1} (compute_pdf_social_learning,
 * social_learning_dynamics.jl:98-114) and HR.  res = {ξ, τ̄_IN, τ̄_OUT, AW_max, tol};
 * t / G / aw_old hold `cap` doubles; SBR_EARG if the knots do not fit. */
int sbr_social_point_paths(sbr_ctx* ctx, double beta, double eta, double x0, double u, double p, double kappa,
                           double lambda, const double* cmp_grid, int32_t n_cmp, double tol, int32_t max_iter,
                           const sbr_opts* opts, double* res, uint32_t* status, int32_t* fp_iters, double* t,
                           double* G, double* aw_old, int64_t cap, int64_t* n_knots);
/* Workspace budget in bytes for social sweeps (0 = 60 % of free HBM at call time). */
int sbr_set_social_workspace(sbr_ctx* ctx, int64_t bytes);
/* Diagnostics: sums over the points of the last social sweep run with
 * SBR_FLAG_DIAG_SOCIAL_PROF — shader cycles in [0] comparison-grid prelude,
 * [1] forced ODE, [2] hazard + crossing scan, [3] bisection, [4] AW norm,
 * [5] damping / AW_max; [6] stage lookups past the register window; [7] RK steps. */
int sbr_social_prof_read(sbr_ctx* ctx, int64_t* out8);
/* Diagnostics of the last social sweep: points promoted into the pool and
 * points re-run from scratch at a larger capacity (either may be NULL). */
int sbr_social_overflow_stats(sbr_ctx* ctx, int64_t* promoted, int64_t* rerun);

/* Interest-rate extension over a β × u grid (one call replaces the loop over
 *     lr = solve_learning(ModelParametersInterest(β_i, η_i, tspan = (0, t_end_i), …).learning)
 *     r  = solve_equilibrium_interest(lr, econ(u_j, p, κ, λ, r, δ), model)
 *                                          interest_rate_solver.jl:51-150
 *     get_AW_functions_interest!(r).AW_max  interest_rate_solver.jl:163-184
 * ): with r > 0 every point integrates the value function
 *     dV/dτ̄ = (HR(τ̄) + δ)(1 − V) + max(u + rV − HR(τ̄), 0),  V(0) = (u+δ)/(r+δ)
 * (value_function_solver.jl:66-112; Tsit5, reltol = abstol = opts->ode_reltol/abstol,
 * saved on the HR grid by the method's dense output) and takes its buffers from
 * h − rV > u; r = 0 is the baseline sweep.  Result layout and status bits as
 * sbr_sweep_baseline (no early-exit post-pass); rk_steps (may be NULL) = value-
 * function Tsit5 steps per point.  SBR_EARG unless 0 <= r < delta
 * (interest_rate_model.jl:48-50).  Host pointers; synchronous. */
int sbr_sweep_interest(sbr_ctx* ctx, const double* beta, const double* eta, const double* t_end, double x0,
                       const double* u, int64_t n_beta, int64_t n_u, double p, double kappa, double lambda, double r,
                       double delta, const sbr_opts* opts, sbr_result_soa* out, int64_t* rk_steps);
/* Same on device pointers, enqueued on `stream`. */
int sbr_sweep_interest_dev(sbr_ctx* ctx, void* stream, const double* beta, const double* eta, const double* t_end,
                           double x0, const double* u, int64_t n_beta, int64_t n_u, double p, double kappa,
                           double lambda, double r, double delta, const sbr_opts* opts, sbr_result_soa* out,
                           int64_t* rk_steps);

/* One interest-rate equilibrium with the paths scripts/3_interest_rates.jl
 * plots (value_function.pdf, hazard_decomposition.pdf): τ̄ grid and HR (n_tau),
 * V on that grid (n_v; 0 when r = 0, fewer than n_tau if the value-function
 * solve stopped early) and AW_cum on the grid (NaN without a run).
 * res = {ξ, τ̄_IN, τ̄_OUT, AW_max, tol}; arrays hold `cap` doubles. */
int sbr_interest_point_paths(sbr_ctx* ctx, double beta, double eta, double t_end, double x0, double u, double p,
                             double kappa, double lambda, double r, double delta, const sbr_opts* opts, double* res,
                             uint32_t* status, double* tau, double* hr, double* V, double* aw_cum, int64_t cap,
                             int64_t* n_tau, int64_t* n_v);

/* 5-consecutive-no-run early exit (1_baseline.jl:236-244) as a post-pass on
 * host arrays: points after `threshold` consecutive non-runs in a β column get
 * SBR_SKIPPED_EARLY_EXIT, xi = aw_max = NaN, tol = Inf. */
void sbr_apply_early_exit(int64_t n_beta, int64_t n_u, int32_t threshold, sbr_result_soa* r);

/* Kernel timing with HIP events recorded on the launch stream around the
 * learning and equilibrium kernels of every baseline sweep call while
 * enabled; sbr_timing_read synchronises `stream` (NULL = the HIP null stream),
 * returns the summed milliseconds per kernel and the number of calls, and
 * resets the accumulators.  A pipelined batch times each learning group's equilibrium
 * launches as one span (first start to last end, the gaps between them included) that counts
 * as that many calls.  This and the other per-device diagnostics below
 * (sbr_learn_stats, sbr_hetero_learn_stats, sbr_social_prof_read,
 * sbr_social_overflow_stats) return SBR_EARG on an n-device context: call them
 * on sbr_multi_child(ctx, rank). */
int sbr_timing_enable(sbr_ctx* ctx, int on);
/* The schedule the last single sweep (sbr_sweep_baseline[_dev]) on this device took: 1 = the
 * per-column readiness schedule (SBR_FLAG_READY_SWEEP granted), 0 = the chunked default (also
 * when the flag was given but the device could not run it: fewer than 256 CUs, or stream
 * creation failed). */
int sbr_last_schedule(sbr_ctx* ctx, int32_t* schedule);
/* Phases of the last host-pointer sbr_sweep_baseline made while timing is enabled, in ms:
 * [0] H2D of the inputs, [1] the kernels (learning, hazard, equilibria), [2] D2H of the results
 * into pinned memory (HIP events on the call's stream), [3] the host side after the sync: the copy
 * into the caller's arrays and the early-exit post-pass, [4] the whole call (host clock; the rest
 * is launch and synchronisation overhead).  On an n-device context (any host-pointer sweep,
 * host clock, timing need not be enabled): [0] the slowest rank's staging + sweep, [1] the
 * slowest rank's D2H into its landing buffer, [2] the host copy into the caller's arrays (or the
 * RCCL gather + scatter), [3] 0, [4] the whole fan-out. */
int sbr_host_phases(sbr_ctx* ctx, double* ms5);
/* Timeline of the last chunked single sweep made while timing is enabled: for each of the
 * *n_chunks column chunks, ms[2k] = its learning end and ms[2k+1] = its equilibrium end, in ms
 * from the sweep start (synchronises `stream` and the learning streams; *n_chunks = 0 when the
 * last sweep was not chunked or not timed).  ms holds 2 × 3 doubles. */
int sbr_chunk_timeline(sbr_ctx* ctx, void* stream, int32_t* n_chunks, double* ms);
int sbr_timing_read(sbr_ctx* ctx, void* stream, double* learn_ms, double* eq_ms, int32_t* n_calls);

/* Per-β learning statistics of the last sweep (knots stored, τ̄-grid length,
 * accepted / rejected RK steps, learning status bits) for flop accounting. */
int sbr_learn_stats(sbr_ctx* ctx, int64_t n_beta, int32_t* n_knots, int32_t* n_tau, int32_t* n_accept,
                    int32_t* n_reject, uint32_t* status);

/* Same for the heterogeneity learning of the last hetero sweep (single-workspace calls:
 * sbr_sweep_hetero[_dev]; the batch pipeline's slot 0 otherwise). */
int sbr_hetero_learn_stats(sbr_ctx* ctx, int64_t n_col, int32_t* n_knots, int32_t* n_tau, int32_t* n_accept,
                           int32_t* n_reject, uint32_t* status);

/* Device facts the engine sized itself with: LDS bytes per workgroup, knots
 * staged in LDS per β column, compute units. */
int sbr_device_info(sbr_ctx* ctx, int32_t* lds_bytes_per_block, int32_t* lds_knot_capacity, int32_t* cu_count);

/* Diagnostics of the n-device data movement without GPUs: the same
 * plan, cyclic column deal, per-rank packing, gather to rank 0 and strided scatter as an
 * sbr_init_multi sweep (csrc/sbr_shard.h), with a host loopback in place of RCCL and the
 * caller's `compute` in place of each rank's GPU sweep.  compute(user, rank, n_cols,
 * col_ids, fields) fills, for the grid columns col_ids[0..n_cols), field f at fields[f] as
 * [n_cols][n_u][per_pt[f]] elements of esz[f] bytes; the scattered results land in
 * host_out[f] (n_col·n_u·per_pt[f] elements, u-fastest per column, NULL = dropped). */
typedef int (*sbr_shard_compute_fn)(void* user, int32_t rank, int64_t n_cols, const int64_t* col_ids,
                                    void* const* fields);
/* rccl_gather = 0: the direct transport (each rank scatters its own block); 1: the gather to rank
 * 0 and one scatter from there (SBR_FLAG_RCCL_GATHER's data movement). */
int sbr_shard_host_run(int32_t n_ranks, int64_t n_col, int64_t n_u, int32_t n_fields, const int64_t* esz,
                       const int64_t* per_pt, void* const* host_out, sbr_shard_compute_fn compute, void* user,
                       int32_t rccl_gather);

/* Diagnostics: sbr_exp / sbr_log / sbr_pow_pos (include/sbr_detmath.h)
 * evaluated on the device, for host/device bit-equality tests. */
int sbr_selftest_detmath(sbr_ctx* ctx, const double* x, const double* y, int n, double* exp_out, double* log_out,
                         double* pow_out);
/* Diagnostics: FastPower.fastpower(x, y) (include/sbr_detmath.h sbr_fastpow, the PI
 * controller's Float32 power) evaluated on the device. */
int sbr_selftest_fastpow(sbr_ctx* ctx, const double* x, const double* y, int n, double* out);

#ifdef __cplusplus
}
#endif

#endif /* SBR_H */
