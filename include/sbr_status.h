/*
 * sbr_status.h — per-point status bits shared by the C-ABI (include/sbr.h),
 * the HIP kernels and the CPU oracle.
 *
 * The reference encodes outcomes as Bool fields plus NaN/Inf sentinels on
 * SolvedModel (src/baseline/solver.jl:55-109, 429-455) and aborts the whole
 * script on exceptions (ArgumentError in model.jl:31-35,71-76; BoundsError
 * from Interpolations' Throw() extrapolation).  A batched engine cannot
 * abort a 4M-point sweep for one point, so every such outcome is a bit here.
 * xi is NaN and tol is Inf whenever SBR_RUN is clear, exactly as in the
 * reference.
 */
#ifndef SBR_STATUS_H
#define SBR_STATUS_H

#define SBR_RUN                 0x0001u /* bankrun == true (solver.jl:452)                    */
#define SBR_CONVERGED           0x0002u /* converged == true (solver.jl:432,453)               */
#define SBR_NO_RUN_HR_BELOW_U   0x0004u /* tau_in == tau_out, trivial no-run (solver.jl:429)   */
#define SBR_NO_RUN_COLLAPSE     0x0008u /* bisection interval collapsed (solver.jl:316)        */
#define SBR_NO_RUN_MAXITER      0x0010u /* bisection iteration cap (solver.jl:321)             */
#define SBR_FALSE_EQ            0x0020u /* root on decreasing branch (solver.jl:354-362)       */
#define SBR_HETERO_INVALID      0x0040u /* is_valid_equilibrium_hetero false (hetero :245)     */
#define SBR_OOB                 0x0080u /* reference would raise BoundsError                   */
#define SBR_SKIPPED_EARLY_EXIT  0x0100u /* 5-consecutive-NaN rule (1_baseline.jl:236-244)      */
#define SBR_ODE_MAXITERS        0x0200u /* integrator hit maxiters (default 1e6, see below)    */
#define SBR_ARG_INVALID         0x0400u /* parameter validation failed (model.jl:31-35,71-76)  */
#define SBR_STIFF_SWITCH        0x0800u /* AutoSwitch moved to Rosenbrock23 (handled, info)   */
#define SBR_SOCIAL_NOT_CONVERGED 0x1000u /* fixed point hit max_iter / stopped (social :390)   */
#define SBR_KNOT_OVERFLOW       0x2000u /* engine knot capacity exceeded (engine limit)        */
#define SBR_ODE_FAILED          0x4000u /* non-finite step size / state                        */
#define SBR_ENGINE_TRUNC        0x8000u /* engine bug: lookup past a truncated knot grid       */
#define SBR_ENGINE_SCHED       0x10000u /* engine bug: a readiness-schedule workgroup timed out
                                            waiting; every point of that sweep is unsolved     */

/* OrdinaryDiffEqCore __init: maxiters = anyadaptive(alg) ? 1000000 : typemax(Int).
 * Every loop iteration (accepted or rejected step) counts. */
#define SBR_DEFAULT_ODE_MAXITERS 1000000

#endif /* SBR_STATUS_H */
