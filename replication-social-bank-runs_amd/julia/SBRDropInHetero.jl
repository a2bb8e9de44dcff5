#=
SBRDropInHetero.jl — drop-in replacement for
src/extensions/heterogeneity/heterogeneity_learning.jl + heterogeneity_solver.jl, backed by
libsbr (the MI355X engine), with the reference's names, argument lists and result structs.

scripts/2_heterogeneity.jl switches by include (INTEGRATION.md §"Extension scripts"):
keep model.jl, plotting.jl and heterogeneity_model.jl (parameter structs and the
LearningResultsHetero / SolvedModelHetero result structs, heterogeneity_model.jl:195-294),
replace learning.jl + solver.jl by SBRDropIn.jl and heterogeneity_learning.jl +
heterogeneity_solver.jl by this file.  Then :59, :67 and :76 run unchanged:

  * `solve_SInetwork_hetero(lp)` → LearningResultsHetero (heterogeneity_learning.jl:49-94):
    the shared knot grid and the K group CDFs of the coupled AutoTsit5(Rosenbrock23()) solve
    at eps() (sbr_learn_hetero), the PDFs by compute_pdf_hetero (:114-134);
  * `solve_equilibrium_hetero(lr, econ; verbose)` → SolvedModelHetero
    (heterogeneity_solver.jl:241-293): per-group buffers, ξ of compute_ξ_hetero with its
    validity check, bankrun / converged / tolerance — one GPU solve on lr's own knot grid
    and group CDFs through sbr_hetero_equilibrium_on_knots (no learning ODE; knots and
    hazards stay resident across the script's per-u calls); HRs are the engine's HR_k on
    hazard_rate's explicit grid (:255);
  * `get_AW_functions_hetero!(result)` → (AW_cum, AW_OUT_groups, AW_IN_groups, AW_groups,
    AW_max) (:386-402 / get_AW_hetero :316-375): every curve comes from the engine — AW_cum and
    AW_max from its AW_total path, AW_OUT_k / AW_IN_k from its per-group rows (AW_k = their
    difference, as :358 forms it), all on lr.grid.

A β×u (or βs-column × u) grid is one call: `SBREngine.solve_equilibrium_hetero_grid`.

NOT EXECUTED IN THIS REPOSITORY (no Julia in the image): the same entry points run through
the Python binding (sbr.learn_hetero / hetero_point_paths, tests/test_hetero.py), and
tests/test_julia_shim.py checks this file's call surface against the reference's
(tests/golden/julia_surface.json, made by tools/extract_julia_surface.py).
=#
using Interpolations

# heterogeneity_learning.jl:114-134 — g_k = (1 − G_k)·β_k·ω with ω = Σ_j dist_j G_j, on the knots
function compute_pdf_hetero(βs, dist, learning_cdfs, t_values)
    Gm = reduce(hcat, [cdf.(t_values) for cdf in learning_cdfs])   # n × K
    # ω as the reference's `sum(dist[j] * I_t[j] for j in 1:K)` (:124): a left fold from the
    # first term, not a BLAS gemv, so every knot sees the same roundings
    ω = dist[1] .* Gm[:, 1]
    for j in 2:length(dist)
        ω = ω .+ dist[j] .* Gm[:, j]
    end
    return Any[LinearInterpolation(t_values, (1 .- Gm[:, k]) .* βs[k] .* ω) for k in eachindex(βs)]
end

# heterogeneity_learning.jl:49-94
function solve_SInetwork_hetero(params::LearningParametersHetero; tol = eps())
    solve_start = time()
    params.tspan[1] == 0 || throw(ArgumentError("the engine integrates from t = 0"))
    # reltol = abstol = tol (heterogeneity_learning.jl:74)
    t, Gm, _ = SBREngine.learn_hetero(sbr_context(), params.βs, params.dist, params.tspan[2], params.x0; tol)
    cdfs = Any[LinearInterpolation(t, Gm[:, k]) for k in eachindex(params.βs)]
    pdfs = compute_pdf_hetero(params.βs, params.dist, cdfs, t)
    return LearningResultsHetero(params, cdfs, pdfs, t, time() - solve_start, nothing)
end

# heterogeneity_solver.jl:316-375 from the engine's paths on lr.grid: `r` is what
# SBREngine.hetero_equilibrium_on_knots returned for this result (AW_total, AW_OUT, AW_IN)
function _get_AW_hetero(result::SolvedModelHetero, r)
    result.bankrun || return nothing
    t_grid = result.learning_results.grid
    K = size(r.AW_OUT, 2)
    outs = Any[LinearInterpolation(t_grid, r.AW_OUT[:, k]) for k in 1:K]
    ins = Any[LinearInterpolation(t_grid, r.AW_IN[:, k]) for k in 1:K]
    nets = Any[LinearInterpolation(t_grid, r.AW_OUT[:, k] .- r.AW_IN[:, k]) for k in 1:K]
    return (AW_cum = LinearInterpolation(t_grid, r.AW_total), AW_OUT_groups = outs, AW_IN_groups = ins,
            AW_groups = nets, AW_max = maximum(r.AW_total))
end

# heterogeneity_solver.jl:316-375 for a SolvedModelHetero built elsewhere: one engine call on its
# learning results' knots (the equilibrium is re-solved on the GPU, its paths returned)
function get_AW_hetero(result::SolvedModelHetero)
    result.bankrun || return nothing
    lr = result.learning_results
    lp = lr.params
    econ = result.model_params.economic
    Gm = reduce(hcat, [cdf.itp.coefs for cdf in lr.learning_cdfs])
    r = SBREngine.hetero_equilibrium_on_knots(sbr_context(), collect(Float64, lr.grid), Gm, lp.βs, lp.dist,
                                              econ.u; η = econ.η, tspan_end = lp.tspan[2], p = econ.p, κ = econ.κ,
                                              λ = econ.λ)
    return _get_AW_hetero(result, r)
end

# heterogeneity_solver.jl:241-293 — one GPU solve on lr_hetero's own knots and group CDFs
# (hazards, buffers, compute_ξ_hetero, validity, AW path); no learning ODE
function solve_equilibrium_hetero(lr_hetero::LearningResultsHetero, econ::EconomicParameters; verbose = false)
    solve_start = time()
    lp = lr_hetero.params
    Gm = reduce(hcat, [cdf.itp.coefs for cdf in lr_hetero.learning_cdfs])   # n × K, on lr_hetero.grid
    r = SBREngine.hetero_equilibrium_on_knots(sbr_context(), collect(Float64, lr_hetero.grid), Gm, lp.βs, lp.dist,
                                              econ.u; η = econ.η, tspan_end = lp.tspan[2], p = econ.p, κ = econ.κ,
                                              λ = econ.λ)
    (r.status & SBREngine.SBR_OOB) != 0 && throw(BoundsError(lr_hetero.learning_cdfs[1], econ.η))
    # the reference's HRs (:255): hazard_rate per group on its explicit grid, from the engine
    HRs = Any[LinearInterpolation(r.τ_bar, r.HR[:, k]) for k in eachindex(lp.βs)]
    bankrun = (r.status & SBREngine.SBR_RUN) != 0
    converged = (r.status & SBREngine.SBR_CONVERGED) != 0
    result = SolvedModelHetero(r.ξ, r.τ_bar_IN_UNCs, r.τ_bar_OUT_UNCs, HRs, bankrun, econ, lr_hetero, converged,
                               time() - solve_start, r.tolerance)
    bankrun && (result.aw[] = _get_AW_hetero(result, r))
    verbose && println(bankrun ? "Converged: ξ = $(result.ξ), tolerance = $(result.tolerance)" :
                                 "No valid run equilibrium exists (status 0x$(string(r.status, base = 16)))")
    return result
end

# heterogeneity_solver.jl:386-402
function get_AW_functions_hetero!(result::SolvedModelHetero)
    result.aw[] !== nothing && return result.aw[]
    result.aw[] = result.bankrun ? get_AW_hetero(result) : nothing
    return result.aw[]
end
