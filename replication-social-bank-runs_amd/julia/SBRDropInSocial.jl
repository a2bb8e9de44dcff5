#=
SBRDropInSocial.jl — drop-in replacement for
src/extensions/social_learning/social_learning_dynamics.jl + social_learning_solver.jl,
backed by libsbr (the MI355X engine), with the reference's names and result structs.

scripts/4_social_learning.jl switches by include (INTEGRATION.md §"Extension scripts"):
keep model.jl and plotting.jl, replace learning.jl + solver.jl by SBRDropIn.jl and
social_learning_dynamics.jl + social_learning_solver.jl by this file.  Then :55-56 (and the
baseline comparison :68-69, :88-89, the plots :104-118) run unchanged:

  * `solve_equilibrium_social_learning(m; tol, max_iter, verbose)` → the SolvedModel of the
    last inner equilibrium (social_learning_solver.jl:63-263, returned at :262): the whole
    damped fixed point (forced Tsit5 learning, baseline equilibrium, get_AW, ∞-norm on
    range(0, η, 1000)) runs on the GPU through sbr_social_point_paths (bit-identical to a
    sweep point).  Its learning_results hold the last iterate's learning_cdf on its knots and
    learning_pdf = (1 − G)·β·AW_{n-1} (compute_pdf_social_learning, dynamics.jl:98-114, from
    the AW_{n-1} the engine returns); HR (solver.jl:424) and get_AW's paths come from the engine
    too (sbr_equilibrium_on_knots_pdf on those knots and pdf values, bit-identical to the
    social point's own inner equilibrium), so `get_AW_functions!(result)` (SBRDropIn.jl) returns
    the engine's AW_cum / AW_OUT / AW_IN (solver.jl:553-576) with no host recomputation.
A β×u grid of fixed points is one call: `SBREngine.solve_equilibrium_social_learning_grid`.

NOT EXECUTED IN THIS REPOSITORY (no Julia in the image): the same entry point runs through
the Python binding (sbr.social_point_paths, tests/test_gpu_social.py), and
tests/test_julia_shim.py checks this file's call surface against the reference's.
=#
using Interpolations

# social_learning_dynamics.jl:132-146 (declared by the reference, unused by its solver)
struct LearningResultsSocial
    params
    learning_cdf::Any
    learning_pdf::Any
    grid::Vector{Float64}
    AW_cum::Any
    solve_time::Float64
    iterations::Int
    converged::Bool
end

# social_learning_dynamics.jl:98-114 — g = (1 − G)·β·AW(t) on t_values
compute_pdf_social_learning(β, learning_cdf, AW_cum, t_values) =
    LinearInterpolation(t_values, (1 .- learning_cdf.(t_values)) .* β .* AW_cum.(t_values))

# social_learning_solver.jl:63-263 — the whole fixed point on the GPU
function solve_equilibrium_social_learning(model::ModelParameters; tol = 1e-4, max_iter = 250, verbose = false,
                                           init_out = 0.0, learning_tol = 1e-12)
    solve_start = time()
    β = model.learning.β
    x0 = model.learning.x0[1]
    econ = model.economic
    η = econ.η
    r = SBREngine.solve_social_point_paths(sbr_context(), β, econ.u; η = η, x0 = x0, p = econ.p, κ = econ.κ,
                                           λ = econ.λ, tol = tol, max_iter = max_iter)
    # the reference raises where an interpolant is read past (0, η) (status SBR_OOB)
    (r.status & SBREngine.SBR_OOB) != 0 && throw(BoundsError(LinearInterpolation(r.t, r.G), η))
    cdf = LinearInterpolation(r.t, r.G)
    g = ((1 .- r.G) .* β) .* r.AW_old
    pdf = LinearInterpolation(r.t, g)
    lr = LearningResults(LearningParameters(β, (0.0, η), x0), cdf, pdf, r.t, 0.0, nothing)
    # the last inner equilibrium's HR and get_AW paths from the engine (sbr_equilibrium_on_knots_pdf
    # on the last iterate's knots and pdf: the social point's ξ, HR and AW, bit for bit)
    e = SBREngine.equilibrium_on_knots(sbr_context(), r.t, r.G, β, econ.u; η = η, tspan_end = η, p = econ.p,
                                       κ = econ.κ, λ = econ.λ, pdf = g)
    HR = LinearInterpolation(e.τ_bar, e.HR)
    bankrun = (r.status & SBREngine.SBR_RUN) != 0
    converged = (r.status & SBREngine.SBR_CONVERGED) != 0
    aw_engine = bankrun ? (AW_cum = e.AW_cum, AW_OUT = e.AW_OUT, AW_IN = e.AW_IN, AW_max = e.AW_max) : nothing
    result = SolvedModel(r.ξ, r.τ_bar_IN_UNC, r.τ_bar_OUT_UNC, HR, bankrun, econ, lr, converged,
                         time() - solve_start, r.tolerance, aw_engine)
    if verbose
        fp_ok = (r.status & SBREngine.SBR_SOCIAL_NOT_CONVERGED) == 0
        println("  Social learning: $(r.fp_iters) fixed-point iterations, converged = $fp_ok")
        println("  Final result: ξ = $(bankrun ? round(result.ξ, digits=3) : "No run")")
    end
    return result
end
