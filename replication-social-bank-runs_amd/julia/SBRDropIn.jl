#=
SBRDropIn.jl — drop-in replacement for src/baseline/learning.jl + src/baseline/solver.jl
backed by libsbr (the MI355X engine), with the reference's names, structs and semantics.

scripts/1_baseline.jl switches with one line: keep

    include(joinpath(@__DIR__, "..", "src", "baseline", "model.jl"))       # parameter structs

and replace the learning.jl / solver.jl includes by

    include(joinpath(@__DIR__, "..", "replication-social-bank-runs_amd", "julia", "SBRDropIn.jl"))

Then Figs 1–3 run unchanged:
  * `solve_learning(lp)`                    → LearningResults (learning.jl:74-81, 109-124): the
    GPU knot grid of AutoTsit5(Rosenbrock23()) at eps() (sbr_learn_baseline), the CDF and
    the symbolic PDF βG(1−G) (compute_pdf_symbolic_baseline, learning.jl:161-173) as
    LinearInterpolations;
  * `solve_equilibrium_baseline(lr, econ)`  → SolvedModel (solver.jl:55-109, 413-462): ξ, the
    buffers, HR as a LinearInterpolation on τ̄, bankrun / converged / tolerance — one GPU
    solve on `lr`'s own knots through sbr_equilibrium_on_knots (no learning ODE: the scripts
    learn once per β, 1_baseline.jl:44 / :227, and call this per u, :169 / :248; the knots
    and HR stay on the GPU between those calls, so each uploads only u);
  * `get_AW_functions!(result)`             → (AW_cum, AW_OUT, AW_IN, AW_max) (solver.jl:553-576):
    all four from the engine (the same call returned get_AW's three paths);
  * `hazard_rate`, `get_AW`                 → host restatements of solver.jl:153-185, 495-532,
    kept for plot_hazard_rate_decomposition / plot_equilibrium (plotting.jl:62-210), which
    call them on interpolants; they are presentation code, not the sweep path.
The extension scripts add their own drop-in on top of this one (they call these too):
SBRDropInHetero.jl (scripts/2_heterogeneity.jl), SBRDropInInterest.jl
(scripts/3_interest_rates.jl), SBRDropInSocial.jl (scripts/4_social_learning.jl); see
INTEGRATION.md for the include lines of each script.
The Fig 4 / Fig 5 loops can keep calling these per point, or call
`SBREngine.solve_equilibrium_grid` once per grid (one ccall per grid, all GPUs of a
`SBREngine.Context(; n_gpus = 8)`).

Differences a caller can see: `LearningResults.ode_solution` is `nothing` (the engine returns
the knots, not an ODESolution); `ξ_guess` is compute_ξ's first iterate as in the reference;
`tol` of `solve_learning` must be `nothing` / `eps()` (the engine integrates at eps()).

NOT EXECUTED IN THIS REPOSITORY: the build image has no Julia.  The same entry points are
exercised through the Python binding (sbr/engine.py: solve_learning,
solve_equilibrium_baseline, get_AW_functions), and tests/test_julia_shim.py checks this file's
struct layouts against include/sbr.h.
=#
using Interpolations

include(joinpath(@__DIR__, "SBREngine.jl"))
using .SBREngine

const _SBR_CTX = Ref{Any}(nothing)
"""The engine context the drop-ins use (one GPU; set `_SBR_CTX[] = SBREngine.Context(; n_gpus = 8)`
to sweep over a node)."""
sbr_context() = (_SBR_CTX[] === nothing && (_SBR_CTX[] = SBREngine.Context()); _SBR_CTX[])

# learning.jl:74-81
struct LearningResults
    params::LearningParameters
    learning_cdf::Any
    learning_pdf::Any
    grid::Vector{Float64}
    solve_time::Float64
    ode_solution::Any   # reference: ODESolution; the engine keeps only the knots (nothing here)
end

# learning.jl:161-173: g = β G (1 − G) on the knots
function compute_pdf_symbolic_baseline(β, learning_cdf, t_values = nothing)
    t_values === nothing && (t_values = learning_cdf.itp.knots[1])
    G_vals = learning_cdf.(t_values)
    return LinearInterpolation(t_values, β .* G_vals .* (1 .- G_vals))
end

# learning.jl:109-124
function solve_learning(learning_params::LearningParameters; tol = nothing)
    solve_start = time()
    learning_params.tspan[1] == 0 || throw(ArgumentError("the engine integrates from t = 0"))
    # solve_SIhomogeneous(…; tol): reltol = abstol = tol, eps() when nothing (learning.jl:41-51)
    t, G, _ = SBREngine.learn(sbr_context(), learning_params.β, learning_params.tspan[2], learning_params.x0;
                              tol = tol === nothing ? eps() : tol)
    cdf = LinearInterpolation(t, G)
    pdf = compute_pdf_symbolic_baseline(learning_params.β, cdf, t)
    return LearningResults(learning_params, cdf, pdf, t, time() - solve_start, nothing)
end

# solver.jl:55-109 (fields, derived τ_IN / τ_OUT, validation and the AW cache as in the reference)
struct SolvedModel
    ξ::Float64
    τ_bar_IN_UNC::Float64
    τ_bar_OUT_UNC::Float64
    HR::Any
    bankrun::Bool
    τ_IN::Float64
    τ_OUT::Float64
    model_params::ModelParameters
    learning_results::LearningResults
    converged::Bool
    solve_time::Float64
    tolerance::Float64
    aw::Ref{Union{Nothing, NamedTuple}}
    aw_engine::Any   # the engine's (AW_cum, AW_OUT, AW_IN, AW_max) on the HR grid (nothing without a run)

    function SolvedModel(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, bankrun, model_params::ModelParameters,
                         learning_results, converged, solve_time, tolerance, aw_engine = nothing)
        τ_IN = max(ξ - τ_bar_IN_UNC, 0)
        τ_OUT = max(ξ - τ_bar_OUT_UNC, 0)
        (ξ ≥ 0 || isnan(ξ)) || throw(ArgumentError("Crash time ξ must be non-negative or NaN, got ξ = $ξ"))
        τ_bar_IN_UNC ≥ 0 || throw(ArgumentError("τ_bar_IN_UNC must be non-negative, got $τ_bar_IN_UNC"))
        τ_bar_OUT_UNC ≥ 0 || throw(ArgumentError("τ_bar_OUT_UNC must be non-negative, got $τ_bar_OUT_UNC"))
        solve_time ≥ 0 || throw(ArgumentError("Solve time must be non-negative, got $solve_time"))
        tolerance ≥ 0 || throw(ArgumentError("Tolerance must be non-negative, got $tolerance"))
        new(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, bankrun, τ_IN, τ_OUT, model_params, learning_results, converged,
            solve_time, tolerance, Ref{Union{Nothing, NamedTuple}}(nothing), aw_engine)
    end

    function SolvedModel(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, bankrun, econ::EconomicParameters,
                         learning_results::LearningResults, converged, solve_time, tolerance, aw_engine = nothing)
        model_params = ModelParameters(learning_results.params, econ)
        return SolvedModel(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, bankrun, model_params, learning_results, converged,
                           solve_time, tolerance, aw_engine)
    end
end

# solver.jl:413-462 — one point on the GPU on learning_results' own knots (hazard, buffers,
# compute_ξ, get_AW's paths); no learning ODE
function solve_equilibrium_baseline(learning_results::LearningResults, econ::EconomicParameters;
                                    ξ_guess = nothing, verbose = false)
    solve_start = time()
    lp = learning_results.params
    cdf = learning_results.learning_cdf
    r = SBREngine.equilibrium_on_knots(sbr_context(), cdf.itp.knots[1], cdf.itp.coefs, lp.β, econ.u; η = econ.η,
                                       tspan_end = lp.tspan[2], p = econ.p, κ = econ.κ, λ = econ.λ,
                                       ξ_guess = ξ_guess)
    (r.status & SBREngine.SBR_OOB) != 0 && throw(BoundsError(cdf, econ.η))
    HR = LinearInterpolation(r.τ_bar, r.HR)
    bankrun = (r.status & SBREngine.SBR_RUN) != 0
    converged = (r.status & SBREngine.SBR_CONVERGED) != 0
    aw_engine = bankrun ? (AW_cum = r.AW_cum, AW_OUT = r.AW_OUT, AW_IN = r.AW_IN, AW_max = r.AW_max) : nothing
    return SolvedModel(r.ξ, r.τ_bar_IN_UNC, r.τ_bar_OUT_UNC, HR, bankrun, econ, learning_results, converged,
                       time() - solve_start, r.tolerance, aw_engine)
end

# hazard_rate (solver.jl:153-185) for the host-side plots (plotting.jl:62-132 calls it on the
# learning PDF).  The τ̄ grid: the PDF's knots up to η with η appended unless it is the last
# one, or an explicit grid's points up to η with η always appended.  Then the running
# trapezoid of w(τ) = e^{aτ}·pdf(τ) from the first point, and the hazard at each point: its
# numerator (p·e^{aτ})·pdf(τ) over p·∫₀^τ w + (1 − p)·∫₀^η w.  Every product and sum is formed
# in the order the engine's hazard kernels use (the same values to the bit).
function hazard_rate(p, a, learning_pdf, η; grid = nothing)
    pts = isnothing(grid) ? learning_pdf.itp.knots[1] : grid
    τs = Float64[τ for τ in pts if τ <= η]
    (!isnothing(grid) || isempty(τs) || τs[end] != η) && push!(τs, η)
    m = length(τs)
    w = [exp(a * τ) * learning_pdf(τ) for τ in τs]
    acc = zeros(m)
    for i in 2:m
        acc[i] = acc[i-1] + 0.5 * (w[i-1] + w[i]) * (τs[i] - τs[i-1])
    end
    hr = [(p * exp(a * τs[i]) * learning_pdf(τs[i])) / (p * acc[i] + (1 - p) * acc[m]) for i in 1:m]
    return LinearInterpolation(τs, hr)
end

# get_AW (solver.jl:495-532) for plot_equilibrium: on HR's knots, the CDF mass that has
# entered (IN) and left (OUT) the withdrawal window by t, each the learning CDF at
# max(t − ξ + τ_con, 0) and zero where t − ξ + τ_con < 0 (τ_con = min(τ_UNC, ξ), with the
# reference's ≥ / > tie rules), and AW_cum = (OUT − IN) + G(0).  All IN values are evaluated
# before all OUT values, as in the reference (the same BoundsError, if any, comes first).
function get_AW(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, learning_cdf)
    ts = HR.itp.knots[1]
    c_in = τ_bar_IN_UNC >= ξ ? ξ : τ_bar_IN_UNC
    c_out = τ_bar_OUT_UNC > ξ ? ξ : τ_bar_OUT_UNC
    window(t, c) = (s = (t - ξ) + c; g = learning_cdf(s > 0 ? s : 0); s >= 0 ? g : zero(g))
    aw_in = [window(t, c_in) for t in ts]
    aw_out = [window(t, c_out) for t in ts]
    g0 = learning_cdf(0)
    aw_cum = [(aw_out[i] - aw_in[i]) + g0 for i in eachindex(ts)]
    return LinearInterpolation(ts, aw_cum), LinearInterpolation(ts, aw_out), LinearInterpolation(ts, aw_in)
end

# solver.jl:553-576 — the engine's get_AW paths on the HR grid and its AW_max (the same maximum
# over the knots, found by the kernel's bounded scan)
function get_AW_functions!(result::SolvedModel)
    result.aw[] !== nothing && return result.aw[]
    result.bankrun || return result.aw[]
    a = result.aw_engine
    if a === nothing # built without the engine's paths (a SolvedModel constructed by the caller)
        AW_cum, AW_OUT, AW_IN = get_AW(result.ξ, result.τ_bar_IN_UNC, result.τ_bar_OUT_UNC, result.HR,
                                       result.learning_results.learning_cdf)
        result.aw[] = (AW_cum = AW_cum, AW_OUT = AW_OUT, AW_IN = AW_IN, AW_max = maximum(AW_cum.itp.coefs))
        return result.aw[]
    end
    τ = result.HR.itp.knots[1]
    result.aw[] = (AW_cum = LinearInterpolation(τ, a.AW_cum), AW_OUT = LinearInterpolation(τ, a.AW_OUT),
                   AW_IN = LinearInterpolation(τ, a.AW_IN), AW_max = a.AW_max)
    return result.aw[]
end
