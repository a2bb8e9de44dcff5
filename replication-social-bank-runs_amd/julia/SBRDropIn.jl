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
the knots, not an ODESolution); `ξ_guess` must be `nothing` (the reference's default midpoint);
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
    (tol === nothing || tol == eps()) || throw(ArgumentError("the engine integrates at reltol = abstol = eps()"))
    learning_params.tspan[1] == 0 || throw(ArgumentError("the engine integrates from t = 0"))
    t, G, _ = SBREngine.learn(sbr_context(), learning_params.β, learning_params.tspan[2], learning_params.x0)
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
    ξ_guess === nothing || throw(ArgumentError("the engine starts the bisection at the reference's default midpoint"))
    lp = learning_results.params
    cdf = learning_results.learning_cdf
    r = SBREngine.equilibrium_on_knots(sbr_context(), cdf.itp.knots[1], cdf.itp.coefs, lp.β, econ.u; η = econ.η,
                                       tspan_end = lp.tspan[2], p = econ.p, κ = econ.κ, λ = econ.λ)
    (r.status & SBREngine.SBR_OOB) != 0 && throw(BoundsError(cdf, econ.η))
    HR = LinearInterpolation(r.τ_bar, r.HR)
    bankrun = (r.status & SBREngine.SBR_RUN) != 0
    converged = (r.status & SBREngine.SBR_CONVERGED) != 0
    aw_engine = bankrun ? (AW_cum = r.AW_cum, AW_OUT = r.AW_OUT, AW_IN = r.AW_IN, AW_max = r.AW_max) : nothing
    return SolvedModel(r.ξ, r.τ_bar_IN_UNC, r.τ_bar_OUT_UNC, HR, bankrun, econ, learning_results, converged,
                       time() - solve_start, r.tolerance, aw_engine)
end

# solver.jl:153-185 (host; plotting.jl:62-132 evaluates it on the learning PDF)
function hazard_rate(p, a, learning_pdf, η; grid = nothing)
    if isnothing(grid)
        τ_bar = learning_pdf.itp.knots[1][learning_pdf.itp.knots[1] .<= η]
        if length(τ_bar) == 0 || τ_bar[end] != η
            push!(τ_bar, η)
        end
    else
        τ_bar = grid[grid .<= η]
        push!(τ_bar, η)
    end
    eg(t) = exp(a * t) * learning_pdf(t)
    int_0_τ_bar = zeros(length(τ_bar))
    for i in 2:length(τ_bar)
        int_0_τ_bar[i] = int_0_τ_bar[i-1] + 0.5 * (eg(τ_bar[i-1]) + eg(τ_bar[i])) * (τ_bar[i] - τ_bar[i-1])
    end
    int_0_η = int_0_τ_bar[end]
    return LinearInterpolation(τ_bar,
        (p .* exp.(a .* τ_bar) .* learning_pdf.(τ_bar)) ./ (p .* int_0_τ_bar .+ (1 - p) .* int_0_η))
end

# solver.jl:495-532 (host; AW_OUT / AW_IN for plot_equilibrium)
function get_AW(ξ, τ_bar_IN_UNC, τ_bar_OUT_UNC, HR, learning_cdf)
    t_grid = HR.itp.knots[1]
    τ_bar_IN_CON = τ_bar_IN_UNC >= ξ ? ξ : τ_bar_IN_UNC
    τ_bar_OUT_CON = τ_bar_OUT_UNC > ξ ? ξ : τ_bar_OUT_UNC
    grid_IN_trunc = ifelse.(t_grid .- ξ .+ τ_bar_IN_CON .> 0, t_grid .- ξ .+ τ_bar_IN_CON, 0)
    AW_IN = ifelse.(t_grid .- ξ .+ τ_bar_IN_CON .>= 0, learning_cdf(grid_IN_trunc), 0)
    grid_OUT_trunc = ifelse.(t_grid .- ξ .+ τ_bar_OUT_CON .> 0, t_grid .- ξ .+ τ_bar_OUT_CON, 0)
    AW_OUT = ifelse.(t_grid .- ξ .+ τ_bar_OUT_CON .>= 0, learning_cdf(grid_OUT_trunc), 0)
    AW_cum = AW_OUT .- AW_IN
    AW_cum .+= learning_cdf(0)
    return LinearInterpolation(t_grid, AW_cum), LinearInterpolation(t_grid, AW_OUT), LinearInterpolation(t_grid, AW_IN)
end

# solver.jl:553-576 — the engine's get_AW paths on the HR grid and its AW_max (the same maximum
# over the knots, found by the kernel's bounded scan)
function get_AW_functions!(result::SolvedModel)
    result.aw[] !== nothing && return result.aw[]
    result.bankrun || return result.aw[]
    a = result.aw_engine
    if a === nothing # built without the engine's paths (SBRDropInSocial's last inner SolvedModel)
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
