#=
SBREngine.jl — Julia binding of libsbr (include/sbr.h) for the reference's scripts.

Drop-in for the β×u loops of scripts/1_baseline.jl (Fig 4 :151-192, Fig 5 :224-267), the
heterogeneity sweep, the social-learning fixed point and the interest-rate equilibrium over a grid: one `ccall` per grid instead of one solve_learning /
solve_equilibrium_baseline / get_AW_functions! per point.  Plain-pointer C ABI; Julia owns every
array (`GC.@preserve`), the library owns device memory.

NOT EXECUTED IN THIS REPOSITORY: the build image has no Julia.  The Python binding
(replication-social-bank-runs_amd/sbr/_lib.py) calls the same symbols with the same layouts and
is what the tests exercise.
=#
module SBREngine

const libsbr = joinpath(@__DIR__, "..", "lib", "libsbr.so")

# sbr_status.h
const SBR_RUN = UInt32(0x0001)
const SBR_CONVERGED = UInt32(0x0002)
const SBR_SKIPPED_EARLY_EXIT = UInt32(0x0100)
const SBR_OOB = UInt32(0x0080)
const SBR_SOCIAL_NOT_CONVERGED = UInt32(0x1000)

struct Opts            # sbr_opts
    ode_reltol::Float64
    ode_abstol::Float64
    ode_maxiters::Int64
    bisect_max_iters::Int32
    early_exit_nan_run::Int32
    knot_capacity::Int32
    hetero_max_iters::Int32
    flags::Int32
    pad::Int32
    xi_guess::Float64
end
# pad = social knot capacity per buffer (0: library default 98304); xi_guess = compute_ξ's first
# iterate (NaN: the reference's midpoint; equilibrium_on_knots only), flagged by SBR_FLAG_XI_GUESS
const SBR_FLAG_XI_GUESS = Int32(0x8)
# tol = the learning ODE's reltol = abstol (solve_learning(lp; tol), learning.jl:43,109; eps() by default)
Opts(; early_exit = 5, xi_guess = NaN, tol = eps()) =
    Opts(Float64(tol), Float64(tol), 1_000_000, 100, early_exit, 65536, 500,
         isnan(xi_guess) ? Int32(0) : SBR_FLAG_XI_GUESS, 0, Float64(xi_guess))

struct ResultSoA       # sbr_result_soa
    xi::Ptr{Float64}
    tau_in_unc::Ptr{Float64}
    tau_out_unc::Ptr{Float64}
    aw_max::Ptr{Float64}
    tol::Ptr{Float64}
    status::Ptr{UInt32}
    iters::Ptr{Int32}
end

"""
    Context(device = 0)            one MI355X
    Context(; n_gpus = 8)          n GPUs of the node: the sweeps below fan out inside libsbr
                                   (one host thread per GPU, β columns dealt cyclically, each GPU
                                   copying its own columns into the caller's arrays) — same
                                   results as one GPU
"""
mutable struct Context
    ptr::Ptr{Cvoid}
    function Context(device::Integer = 0; n_gpus::Union{Nothing, Integer} = nothing)
        r = Ref{Ptr{Cvoid}}(C_NULL)
        rc = n_gpus === nothing ?
             ccall((:sbr_init, libsbr), Cint, (Cint, Ptr{Ptr{Cvoid}}), device, r) :
             ccall((:sbr_init_multi, libsbr), Cint, (Cint, Ptr{Cint}, Ptr{Ptr{Cvoid}}), n_gpus, C_NULL, r)
        rc == 0 || error("sbr_init failed ($rc): no usable MI355X")
        ctx = new(r[])
        finalizer(c -> ccall((:sbr_free, libsbr), Cint, (Ptr{Cvoid},), c.ptr), ctx)
        return ctx
    end
end

n_gpus(ctx::Context) = Int(ccall((:sbr_multi_size, libsbr), Cint, (Ptr{Cvoid},), ctx.ptr))

function check(ctx::Context, rc)
    rc == 0 && return
    msg = unsafe_string(ccall((:sbr_last_error, libsbr), Cstring, (Ptr{Cvoid},), ctx.ptr))
    rc == -1 ? throw(ArgumentError(msg)) : error("libsbr: $msg ($rc)")
end

"""
    solve_equilibrium_grid(ctx, β_vals, u_vals; η, tspan_end, x0, p, κ, λ, early_exit=5)

Batched `solve_learning` + `solve_equilibrium_baseline` + `get_AW_functions!` for every
(β, u).  `η`/`tspan_end` are per-β (scalars broadcast): the copy-modify constructor of
model.jl:189-211 carries η = 15, tspan = (0, 30) for every β of Fig 5.  Returns
`(max_AW_matrix, ξ, τ̄_IN, τ̄_OUT, status)` as [u, β] matrices — `max_AW_matrix` is the
matrix of scripts/1_baseline.jl:213 (NaN = no run or skipped by the 5-NaN rule).
"""
function solve_equilibrium_grid(ctx::Context, β_vals, u_vals; η = 15.0, tspan_end = 30.0, x0 = 1e-4,
                                p = 0.5, κ = 0.6, λ = 0.01, early_exit = 5)
    β = collect(Float64, β_vals); u = collect(Float64, u_vals)
    nb, nu = length(β), length(u)
    ηv = fill(Float64(η), nb) .+ 0 .* β
    tv = fill(Float64(tspan_end), nb)
    # u-fastest layout [u, β] == Julia's column-major max_AW_matrix[j, i]
    xi = Matrix{Float64}(undef, nu, nb); tin = similar(xi); tout = similar(xi)
    aw = similar(xi); tol = similar(xi); st = Matrix{UInt32}(undef, nu, nb)
    opts = Ref(Opts(; early_exit))
    GC.@preserve β u ηv tv xi tin tout aw tol st begin
        soa = Ref(ResultSoA(pointer(xi), pointer(tin), pointer(tout), pointer(aw), pointer(tol), pointer(st),
                            Ptr{Int32}(C_NULL)))
        rc = ccall((:sbr_sweep_baseline, libsbr), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64, Ptr{Float64}, Int64, Int64,
                    Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA}),
                   ctx.ptr, β, ηv, tv, x0, u, nb, nu, p, κ, λ, opts, soa)
        check(ctx, rc)
    end
    return (max_AW_matrix = aw, ξ = xi, τ_bar_IN_UNC = tin, τ_bar_OUT_UNC = tout, status = st)
end

"""
    learn(ctx, β, tspan_end, x0; cap = 1 << 16)

`solve_SIhomogeneous` (learning.jl:41-54) on the GPU: the knot grid `t` and CDF values `G`
of the adaptive AutoTsit5(Rosenbrock23()) solution on (0, tspan_end), and the status bits.
"""
function learn(ctx::Context, β, tspan_end, x0; cap = 1 << 16, tol = eps())
    t = Vector{Float64}(undef, cap); G = similar(t); nk = Ref{Int32}(0); st = Ref{UInt32}(0)
    b = Float64[β]; e = Float64[tspan_end]; te = Float64[tspan_end]
    opts = Ref(Opts(; early_exit = 0, tol))
    GC.@preserve t G b e te begin
        rc = ccall((:sbr_learn_baseline, libsbr), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64, Int64, Int32, Ref{Opts},
                    Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int32}, Ref{UInt32}),
                   ctx.ptr, b, e, te, x0, 1, Int32(0), opts, t, G, cap, nk, st)
        check(ctx, rc)
    end
    n = Int(nk[])
    return t[1:n], G[1:n], st[]
end

"""
    solve_point_paths(ctx, β, u; η, tspan_end, x0, p, κ, λ, cap = 1 << 16)

One point with paths — `solve_learning` + `solve_equilibrium_baseline` + `get_AW`
(src/baseline/solver.jl:413-462, 495-532) — returning the hazard grid τ̄, HR(τ̄) and AW_cum(τ̄),
from which a maintainer rebuilds the `LinearInterpolation`s the plotting code consumes
(`HR = LinearInterpolation(τ̄, hr)`, `AW_cum = LinearInterpolation(τ̄, aw_cum)`, plotting.jl:156-210).
"""
function solve_point_paths(ctx::Context, β, u; η = 15.0, tspan_end = 30.0, x0 = 1e-4, p = 0.5, κ = 0.6,
                           λ = 0.01, cap = 1 << 16)
    res = zeros(Float64, 5); st = Ref{UInt32}(0); nt = Ref{Int64}(0)
    τ = Vector{Float64}(undef, cap); hr = similar(τ); aw = similar(τ)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve res τ hr aw begin
        rc = ccall((:sbr_solve_point_paths, libsbr), Cint,
                   (Ptr{Cvoid}, Float64, Float64, Float64, Float64, Float64, Float64, Float64, Float64, Ref{Opts},
                    Ptr{Float64}, Ref{UInt32}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                   ctx.ptr, β, η, tspan_end, x0, u, p, κ, λ, opts, res, st, τ, hr, aw, cap, nt)
        check(ctx, rc)
    end
    k = nt[]
    return (ξ = res[1], τ_bar_IN_UNC = res[2], τ_bar_OUT_UNC = res[3], AW_max = res[4], tolerance = res[5],
            status = st[], τ_bar = τ[1:k], HR = hr[1:k], AW_cum = aw[1:k])
end

"""
    equilibrium_on_knots(ctx, t, G, β, u; η, tspan_end, p, κ, λ)

`solve_equilibrium_baseline(lr, econ)` + `get_AW_functions!` (src/baseline/solver.jl:413-462,
495-576) on a LearningResults' own knot grid (`t`, `G` = `lr.learning_cdf`'s knots and values,
`β` = `lr.params.β`, `tspan_end` = `lr.params.tspan[2]`): no learning ODE; `ξ_guess` is
compute_ξ's first iterate (solver.jl:413,441; `nothing` = the midpoint).  The knots and the
hazard path stay on the GPU while `t`, `G`, β, η, p and λ repeat, so the scripts' per-u loops
(1_baseline.jl:169, 248) upload only `u`.  Returns ξ, the buffers, AW_max, the tolerance, the
status and the hazard grid τ̄ with HR(τ̄), AW_cum, AW_OUT and AW_IN on it (NaN without a run).
`pdf`: the learning pdf's values on the knots (sbr_equilibrium_on_knots_pdf; β unused) — the
social extension's (1 − G)·β·AW_{n−1}; `nothing` = βG(1 − G).
"""
function equilibrium_on_knots(ctx::Context, t::Vector{Float64}, G::Vector{Float64}, β, u; η, tspan_end,
                              p = 0.5, κ = 0.6, λ = 0.01, ξ_guess = nothing, pdf = nothing)
    n = length(t)
    length(G) == n || throw(ArgumentError("t and G must have the same length"))
    pdf === nothing || length(pdf) == n || throw(ArgumentError("t and pdf must have the same length"))
    cap = n + 1
    res = fill(NaN, 5); st = UInt32[0]; it = Int32[0]; nt = Ref{Int64}(0)
    τ = Vector{Float64}(undef, cap); hr = similar(τ); cum = similar(τ); awo = similar(τ); awi = similar(τ)
    uv = Float64[u]
    opts = Ref(Opts(; early_exit = 0, xi_guess = ξ_guess === nothing ? NaN : ξ_guess))
    GC.@preserve t G uv res st it τ hr cum awo awi begin
        soa = Ref(ResultSoA(pointer(res, 1), pointer(res, 2), pointer(res, 3), pointer(res, 4), pointer(res, 5),
                            pointer(st), pointer(it)))
        rc = if pdf === nothing
            ccall((:sbr_equilibrium_on_knots, libsbr), Cint,
                  (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Float64, Float64, Float64, Ptr{Float64}, Int64,
                   Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                   Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                  ctx.ptr, t, G, n, β, η, tspan_end, uv, 1, p, κ, λ, opts, soa, τ, hr, cum, awo, awi, cap, nt)
        else
            pv = Vector{Float64}(pdf)
            GC.@preserve pv ccall((:sbr_equilibrium_on_knots_pdf, libsbr), Cint,
                  (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Float64, Float64, Ptr{Float64},
                   Int64, Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA}, Ptr{Float64}, Ptr{Float64},
                   Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                  ctx.ptr, t, G, pv, n, η, tspan_end, uv, 1, p, κ, λ, opts, soa, τ, hr, cum, awo, awi, cap, nt)
        end
        check(ctx, rc)
    end
    k = nt[]
    return (ξ = res[1], τ_bar_IN_UNC = res[2], τ_bar_OUT_UNC = res[3], AW_max = res[4], tolerance = res[5],
            status = st[1], τ_bar = τ[1:k], HR = hr[1:k], AW_cum = cum[1:k], AW_OUT = awo[1:k], AW_IN = awi[1:k])
end

"""
    solve_equilibrium_hetero_grid(ctx, βs_cols, dist, u_vals; η, tspan_end, x0, p, κ, λ)

`βs_cols` is K × n_col (column c = the group rates of one parameter column); η per column.
"""
function solve_equilibrium_hetero_grid(ctx::Context, βs_cols::AbstractMatrix, dist, u_vals; η, tspan_end,
                                       x0 = 1e-4, p = 0.9, κ = 0.3, λ = 0.1)
    B = Matrix{Float64}(βs_cols); K, nc = size(B)
    d = collect(Float64, dist); u = collect(Float64, u_vals); nu = length(u)
    ηv = collect(Float64, η); tv = fill(Float64(tspan_end), nc) .+ 0 .* ηv
    xi = Matrix{Float64}(undef, nu, nc); aw = similar(xi); tol = similar(xi); st = Matrix{UInt32}(undef, nu, nc)
    tin = Array{Float64}(undef, K, nu, nc); tout = similar(tin)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve B d u ηv tv xi aw tol st tin tout begin
        soa = Ref(ResultSoA(pointer(xi), C_NULL, C_NULL, pointer(aw), pointer(tol), pointer(st), C_NULL))
        rc = ccall((:sbr_sweep_hetero, libsbr), Cint,
                   (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64,
                    Ptr{Float64}, Int64, Int64, Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA},
                    Ptr{Float64}, Ptr{Float64}),
                   ctx.ptr, K, B, d, ηv, tv, x0, u, nc, nu, p, κ, λ, opts, soa, tin, tout)
        check(ctx, rc)
    end
    return (AW_max = aw, ξ = xi, τ_bar_IN_UNCs = tin, τ_bar_OUT_UNCs = tout, status = st)
end

"""
    solve_equilibrium_social_learning_grid(ctx, β_vals, u_vals; η, x0, p, κ, λ, tol=1e-4, max_iter=500)

Batched `solve_equilibrium_social_learning(ModelParameters(…); tol, max_iter)`
(src/extensions/social_learning/social_learning_solver.jl:63-263) for every (β, u), plus
`get_AW_functions!(result).AW_max`.  `η` per β (copy-modify carries η = η_bar/β_base as in
scripts/4_social_learning.jl); the comparison grid of :103 is handed over as Julia's own
`collect(range(0.0, η, length = 1000))`.  Returns [u, β] matrices; `fp_iters` = fixed-point
iterations; `status & SBR_SOCIAL_NOT_CONVERGED` marks points the reference leaves unconverged
(or where it would raise a BoundsError: `SBR_OOB`).
"""
function solve_equilibrium_social_learning_grid(ctx::Context, β_vals, u_vals; η, x0 = 1e-4, p = 0.99,
                                                κ = 0.25, λ = 0.25, tol = 1e-4, max_iter = 500)
    β = collect(Float64, β_vals); u = collect(Float64, u_vals)
    nb, nu = length(β), length(u)
    ηv = fill(Float64(η), nb) .+ 0 .* β
    cmp = reduce(hcat, [collect(range(0.0, e, length = 1000)) for e in ηv])   # 1000 × nb, column b = β_b's grid
    xi = Matrix{Float64}(undef, nu, nb); tin = similar(xi); tout = similar(xi)
    aw = similar(xi); tl = similar(xi); st = Matrix{UInt32}(undef, nu, nb)
    fp = Matrix{Int32}(undef, nu, nb); steps = Matrix{Int64}(undef, nu, nb)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve β u ηv cmp xi tin tout aw tl st fp steps begin
        soa = Ref(ResultSoA(pointer(xi), pointer(tin), pointer(tout), pointer(aw), pointer(tl), pointer(st),
                            Ptr{Int32}(C_NULL)))
        rc = ccall((:sbr_sweep_social, libsbr), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Float64, Ptr{Float64}, Int64, Int64, Float64, Float64,
                    Float64, Ptr{Float64}, Int32, Float64, Int32, Ref{Opts}, Ref{ResultSoA}, Ptr{Int32},
                    Ptr{Int64}),
                   ctx.ptr, β, ηv, x0, u, nb, nu, p, κ, λ, cmp, Int32(1000), tol, Int32(max_iter), opts, soa,
                   fp, steps)
        check(ctx, rc)
    end
    return (AW_max = aw, ξ = xi, τ_bar_IN_UNC = tin, τ_bar_OUT_UNC = tout, tolerance = tl, status = st,
            fp_iters = fp, rk_steps = steps)
end

"""
    solve_equilibrium_interest_grid(ctx, β_vals, u_vals; r, δ, η = 15.0, tspan_end = 30.0, x0 = 1e-4,
                                    p = 0.5, κ = 0.6, λ = 0.01)

`solve_learning` + `solve_equilibrium_interest` (interest_rate_solver.jl:51-150) +
`get_AW_functions_interest!(…).AW_max` for every (β_i, u_j), η and tspan carried as in
the Fig 5 copy-modify loop.  Matrices are n_u × n_β; `rk_steps` counts the value
function's Tsit5 steps per point.
"""
function solve_equilibrium_interest_grid(ctx::Context, β_vals, u_vals; r, δ, η = 15.0, tspan_end = 30.0,
                                         x0 = 1e-4, p = 0.5, κ = 0.6, λ = 0.01)
    β = collect(Float64, β_vals); u = collect(Float64, u_vals)
    nb, nu = length(β), length(u)
    ηv = fill(Float64(η), nb); tv = fill(Float64(tspan_end), nb)
    xi = Matrix{Float64}(undef, nu, nb); tin = similar(xi); tout = similar(xi)
    aw = similar(xi); tl = similar(xi); st = Matrix{UInt32}(undef, nu, nb)
    steps = Matrix{Int64}(undef, nu, nb)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve β u ηv tv xi tin tout aw tl st steps begin
        soa = Ref(ResultSoA(pointer(xi), pointer(tin), pointer(tout), pointer(aw), pointer(tl), pointer(st),
                            Ptr{Int32}(C_NULL)))
        rc = ccall((:sbr_sweep_interest, libsbr), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64, Ptr{Float64}, Int64, Int64,
                    Float64, Float64, Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA}, Ptr{Int64}),
                   ctx.ptr, β, ηv, tv, x0, u, nb, nu, p, κ, λ, r, δ, opts, soa, steps)
        check(ctx, rc)
    end
    return (AW_max = aw, ξ = xi, τ_bar_IN_UNC = tin, τ_bar_OUT_UNC = tout, tolerance = tl, status = st,
            rk_steps = steps)
end

"""
    solve_interest_point_paths(ctx, β, u; r, δ, η = 15.0, tspan_end = 30.0, x0 = 1e-4, p = 0.5, κ = 0.6, λ = 0.01)

`solve_equilibrium_interest` for one point with what `scripts/3_interest_rates.jl` plots:
`V = LinearInterpolation(τ_bar[1:length(V)], V)` is the reference's value-function
interpolant (saved on the HR grid), `HR = LinearInterpolation(τ_bar, HR)`.
"""
function solve_interest_point_paths(ctx::Context, β, u; r, δ, η = 15.0, tspan_end = 30.0, x0 = 1e-4, p = 0.5,
                                    κ = 0.6, λ = 0.01, cap = 1 << 16)
    res = zeros(Float64, 5); st = Ref{UInt32}(0); nt = Ref{Int64}(0); nv = Ref{Int64}(0)
    τ = Vector{Float64}(undef, cap); hr = similar(τ); V = similar(τ); aw = similar(τ)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve res τ hr V aw begin
        rc = ccall((:sbr_interest_point_paths, libsbr), Cint,
                   (Ptr{Cvoid}, Float64, Float64, Float64, Float64, Float64, Float64, Float64, Float64, Float64,
                    Float64, Ref{Opts}, Ptr{Float64}, Ref{UInt32}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Int64, Ref{Int64}, Ref{Int64}),
                   ctx.ptr, β, η, tspan_end, x0, u, p, κ, λ, r, δ, opts, res, st, τ, hr, V, aw, cap, nt, nv)
        check(ctx, rc)
    end
    k = nt[]; m = nv[]
    return (ξ = res[1], τ_bar_IN_UNC = res[2], τ_bar_OUT_UNC = res[3], AW_max = res[4], tolerance = res[5],
            status = st[], τ_bar = τ[1:k], HR = hr[1:k], V = V[1:m], AW_cum = aw[1:k])
end

"""
    solve_social_point_paths(ctx, β, u; η, x0 = 1e-4, p = 0.99, κ = 0.25, λ = 0.25, tol = 1e-4, max_iter = 500)

`solve_equilibrium_social_learning` for one point with the learning knots `t`, `G` of the
returned `SolvedModel` and `AW_old` = AW_{n-1}(t) (the forcing that drove that iterate);
`LinearInterpolation(t, G)` is its `learning_cdf`, `(1 .- G) .* β .* AW_old` its
`learning_pdf` (compute_pdf_social_learning), from which `hazard_rate` and `get_AW` rebuild
the curves of `scripts/4_social_learning.jl` (HR grid τ̄ = knots ≤ η, plus η).
"""
function solve_social_point_paths(ctx::Context, β, u; η, x0 = 1e-4, p = 0.99, κ = 0.25, λ = 0.25, tol = 1e-4,
                                  max_iter = 500, cap = 1 << 20)
    cmp = collect(range(0.0, Float64(η), length = 1000))
    res = zeros(Float64, 5); st = Ref{UInt32}(0); fp = Ref{Int32}(0); nk = Ref{Int64}(0)
    t = Vector{Float64}(undef, cap); G = similar(t); awo = similar(t)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve cmp res t G awo begin
        rc = ccall((:sbr_social_point_paths, libsbr), Cint,
                   (Ptr{Cvoid}, Float64, Float64, Float64, Float64, Float64, Float64, Float64, Ptr{Float64}, Int32,
                    Float64, Int32, Ref{Opts}, Ptr{Float64}, Ref{UInt32}, Ref{Int32}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Int64, Ref{Int64}),
                   ctx.ptr, β, η, x0, u, p, κ, λ, cmp, Int32(1000), tol, Int32(max_iter), opts, res, st, fp, t, G,
                   awo, cap, nk)
        check(ctx, rc)
    end
    k = nk[]
    return (ξ = res[1], τ_bar_IN_UNC = res[2], τ_bar_OUT_UNC = res[3], AW_max = res[4], tolerance = res[5],
            status = st[], fp_iters = fp[], t = t[1:k], G = G[1:k], AW_old = awo[1:k])
end

"""
    learn_hetero(ctx, βs, dist, tspan_end, x0; cap = 1 << 14)

`solve_SInetwork_hetero` (heterogeneity_learning.jl:49-94) on the GPU: the shared knot grid
`t` and the group CDFs `G` (n × K) of the coupled AutoTsit5(Rosenbrock23()) solve at eps()
on (0, tspan_end), and the status bits.
"""
function learn_hetero(ctx::Context, βs, dist, tspan_end, x0; cap = 1 << 14, tol = eps())
    b = collect(Float64, βs); d = collect(Float64, dist); K = length(d)
    t = Vector{Float64}(undef, cap); G = Vector{Float64}(undef, cap * K)
    nk = Ref{Int32}(0); st = Ref{UInt32}(0); te = Float64[tspan_end]
    opts = Ref(Opts(; early_exit = 0, tol))
    GC.@preserve b d t G te begin
        rc = ccall((:sbr_learn_hetero, libsbr), Cint,
                   (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Float64, Int64, Ref{Opts},
                    Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int32}, Ref{UInt32}),
                   ctx.ptr, Int32(K), b, d, te, x0, 1, opts, t, G, cap, nk, st)
        check(ctx, rc)
    end
    n = Int(nk[])
    return t[1:n], permutedims(reshape(G[1:n*K], K, n)), st[]
end

"""
    hetero_equilibrium_on_knots(ctx, t, Gm, βs, dist, u; η, tspan_end, p = 0.9, κ = 0.3, λ = 0.1)

`solve_equilibrium_hetero(lr_hetero, econ)` + `get_AW_functions_hetero!`
(heterogeneity_solver.jl:241-293, 316-402) on a LearningResultsHetero's own knot grid `t` and
group CDF values `Gm` (n × K: column k = `learning_cdfs[k]`'s coefficients): no learning ODE.
Knots, CDFs and the K hazard paths stay on the GPU while the inputs repeat.  Returns ξ, the
per-group buffers, AW_max, the tolerance, the status, the hazard grid τ̄ with HR_k(τ̄) as the
columns of `HR` (the reference's `HRs`, :255), `AW_total` on the knots and get_AW_hetero's
per-group curves `AW_OUT` / `AW_IN` (n × K, column k = group k, :335-362) — NaN without a run.
"""
function hetero_equilibrium_on_knots(ctx::Context, t::Vector{Float64}, Gm::AbstractMatrix, βs, dist, u; η, tspan_end,
                                     p = 0.9, κ = 0.3, λ = 0.1)
    n = length(t); K = length(dist)
    size(Gm) == (n, K) || throw(ArgumentError("Gm must be length(t) × length(dist)"))
    Gk = Matrix{Float64}(permutedims(Gm))        # knot-major [n][K] == a K × n column-major matrix
    b = collect(Float64, βs); d = collect(Float64, dist)
    cap = n + 1
    res = fill(NaN, 5); st = UInt32[0]; it = Int32[0]; nt = Ref{Int64}(0)
    tin = zeros(Float64, K); tout = zeros(Float64, K)
    hr = Matrix{Float64}(undef, cap, K); aw = Vector{Float64}(undef, n)
    awg = Matrix{Float64}(undef, cap, 2K)          # columns: AW_OUT_1..K, AW_IN_1..K (stride cap)
    uv = Float64[u]
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve t Gk b d uv res st it tin tout hr aw awg begin
        soa = Ref(ResultSoA(pointer(res, 1), C_NULL, C_NULL, pointer(res, 4), pointer(res, 5), pointer(st),
                            pointer(it)))
        rc = ccall((:sbr_hetero_equilibrium_on_knots, libsbr), Cint,
                   (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Float64,
                    Float64, Ptr{Float64}, Int64, Float64, Float64, Float64, Ref{Opts}, Ref{ResultSoA},
                    Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                   ctx.ptr, Int32(K), t, Gk, n, b, d, η, tspan_end, uv, 1, p, κ, λ, opts, soa, tin, tout, hr, aw,
                   awg, cap, nt)
        check(ctx, rc)
    end
    k = nt[]
    return (ξ = res[1], AW_max = res[4], tolerance = res[5], status = st[1], τ_bar_IN_UNCs = tin,
            τ_bar_OUT_UNCs = tout, τ_bar = k > 0 ? vcat(t[t .<= η], η)[1:k] : Float64[], HR = hr[1:k, :],
            AW_total = aw, AW_OUT = awg[1:n, 1:K], AW_IN = awg[1:n, K+1:2K])
end

"""
    solve_hetero_point_paths(ctx, βs, dist, u; η, tspan_end, x0 = 1e-4, p = 0.9, κ = 0.3, λ = 0.1)

One heterogeneity equilibrium with the learning knots `t`, the group CDFs `G` (n × K), the
per-group buffers, `AW_total` on the knots (`get_AW_functions_hetero!`) and the per-group
curves `AW_OUT` / `AW_IN` (n × K, get_AW_hetero :335-362).
"""
function solve_hetero_point_paths(ctx::Context, βs, dist, u; η, tspan_end, x0 = 1e-4, p = 0.9, κ = 0.3, λ = 0.1,
                                  cap = 1 << 16)
    b = collect(Float64, βs); d = collect(Float64, dist); K = length(d)
    res = zeros(Float64, 3); st = Ref{UInt32}(0); nk = Ref{Int64}(0)
    tin = zeros(Float64, K); tout = zeros(Float64, K)
    t = Vector{Float64}(undef, cap); G = Vector{Float64}(undef, cap * K); aw = similar(t)
    awg = Matrix{Float64}(undef, cap, 2K)
    opts = Ref(Opts(; early_exit = 0))
    GC.@preserve b d res tin tout t G aw awg begin
        rc = ccall((:sbr_hetero_point_paths, libsbr), Cint,
                   (Ptr{Cvoid}, Int32, Ptr{Float64}, Ptr{Float64}, Float64, Float64, Float64, Float64, Float64,
                    Float64, Float64, Ref{Opts}, Ptr{Float64}, Ref{UInt32}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                    Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Int64, Ref{Int64}),
                   ctx.ptr, K, b, d, η, tspan_end, x0, u, p, κ, λ, opts, res, st, tin, tout, t, G, aw, awg, cap, nk)
        check(ctx, rc)
    end
    n = nk[]
    return (ξ = res[1], AW_max = res[2], tolerance = res[3], status = st[], τ_bar_IN_UNCs = tin,
            τ_bar_OUT_UNCs = tout, t = t[1:n], G = permutedims(reshape(G[1:n*K], K, n)), AW_total = aw[1:n],
            AW_OUT = awg[1:n, 1:K], AW_IN = awg[1:n, K+1:2K])
end

end # module
