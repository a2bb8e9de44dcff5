#=
SBRDropInInterest.jl — drop-in replacement for
src/extensions/interest_rates/value_function_solver.jl + interest_rate_solver.jl, backed by
libsbr (the MI355X engine), with the reference's names, argument lists and result structs.

scripts/3_interest_rates.jl switches by include (INTEGRATION.md §"Extension scripts"):
keep model.jl, plotting.jl and interest_rate_model.jl (ModelParametersInterest,
EconomicParametersInterest and the SolvedModelInterest result struct,
interest_rate_model.jl:25-245), replace learning.jl + solver.jl by SBRDropIn.jl and
value_function_solver.jl + interest_rate_solver.jl by this file.  Then :56, :64 and :72 run
unchanged:

  * `solve_learning(m.learning)` (SBRDropIn.jl) → LearningResults;
  * `solve_equilibrium_interest(lr, econ, model; ξ_guess, verbose)` → SolvedModelInterest
    (interest_rate_solver.jl:51-150): HR, the value function V (r > 0: the HJB ODE of
    value_function_solver.jl:66-112 at eps(), saved on the HR grid), the buffers on h − rV,
    the baseline compute_ξ — one GPU solve through sbr_interest_point_paths (bit-identical to a
    sweep point); V is `LinearInterpolation(saved grid, V)` like the reference's (:109);
  * `get_AW_functions_interest!(result)` → (AW_cum, AW_OUT, AW_IN, AW_max) (:161-184): AW_cum
    and AW_max from the engine, AW_OUT / AW_IN rebuilt by `get_AW` (SBRDropIn.jl).
The script's plots then read `result.V`, `result.learning_results.learning_pdf` and call
`hazard_rate(1.0, λ, pdf, η)` (SBRDropIn.jl) as before.  A β×u grid is one call:
`SBREngine.solve_equilibrium_interest_grid`.

NOT EXECUTED IN THIS REPOSITORY (no Julia in the image): the same entry points run through
the Python binding (sbr.interest_point_paths, tests/test_interest.py), and
tests/test_julia_shim.py checks this file's call surface against the reference's.
=#
using Interpolations

# interest_rate_solver.jl:51-150
function solve_equilibrium_interest(lr::LearningResults, econ::EconomicParametersInterest,
                                    model::ModelParametersInterest; ξ_guess = nothing, verbose = false)
    solve_start = time()
    # ξ_guess is accepted and, as in the reference, not used: interest_rate_solver.jl:113 calls
    # compute_ξ(τ̄_IN, τ̄_OUT, learning_cdf, κ; verbose) without it — the bisection starts at the midpoint
    lp = lr.params
    r = SBREngine.solve_interest_point_paths(sbr_context(), lp.β, econ.u; r = econ.r, δ = econ.δ, η = econ.η,
                                             tspan_end = lp.tspan[2], x0 = lp.x0, p = econ.p, κ = econ.κ, λ = econ.λ)
    (r.status & SBREngine.SBR_OOB) != 0 && throw(BoundsError(lr.learning_cdf, econ.η))
    HR = LinearInterpolation(r.τ_bar, r.HR)
    V = econ.r > 0 ? LinearInterpolation(r.τ_bar[1:length(r.V)], r.V) : nothing
    bankrun = (r.status & SBREngine.SBR_RUN) != 0
    converged = (r.status & SBREngine.SBR_CONVERGED) != 0
    result = SolvedModelInterest(r.ξ, r.τ_bar_IN_UNC, r.τ_bar_OUT_UNC, HR, bankrun, V, model, lr, converged,
                                 time() - solve_start, r.tolerance)
    if bankrun
        _, AW_OUT_func, AW_IN_func = get_AW(result.ξ, result.τ_bar_IN_UNC, result.τ_bar_OUT_UNC, HR, lr.learning_cdf)
        result.aw[] = (AW_cum = LinearInterpolation(r.τ_bar, r.AW_cum), AW_OUT = AW_OUT_func, AW_IN = AW_IN_func,
                       AW_max = maximum(r.AW_cum))
    end
    verbose && println(bankrun ? "  Crisis time: ξ=$(round(result.ξ, digits=3))" :
                                 "  No bank run equilibrium (status 0x$(string(r.status, base = 16)))")
    return result
end

# interest_rate_solver.jl:161-184
function get_AW_functions_interest!(result::SolvedModelInterest)
    result.aw[] !== nothing && return result.aw[]
    result.bankrun || return (result.aw[] = nothing)
    AW_cum_func, AW_OUT_func, AW_IN_func = get_AW(result.ξ, result.τ_bar_IN_UNC, result.τ_bar_OUT_UNC, result.HR,
                                                  result.learning_results.learning_cdf)
    result.aw[] = (AW_cum = AW_cum_func, AW_OUT = AW_OUT_func, AW_IN = AW_IN_func,
                   AW_max = maximum(AW_cum_func.itp.coefs))
    return result.aw[]
end
