"""Interest-rate extension (src/extensions/interest_rates/): the CPU restatement
pinned to the committed figures of scripts/3_interest_rates.jl, and the GPU
sweep bit-identical to it."""
import numpy as np
import pytest

import sbr

P = dict(beta=1.0, eta=15.0, t_end=30.0, u=0.0, p=0.5, kappa=0.6, lam=0.01, r=0.06, delta=0.1)


def _script_point(oracle):
    return oracle.interest_point(P["beta"], P["eta"], P["t_end"], P["u"], P["p"], P["kappa"], P["lam"], P["r"],
                                 P["delta"])


def test_interest_value_function_figure(oracle, golden):
    """value_function.pdf: ξ from the drawn sample count and the first sample's offset,
    and V(τ) on range(0, η, 500) (the drawn half, t = ξ − τ ≥ 0)."""
    g = golden("interest_rates.json")["value_function"]
    r = _script_point(oracle)
    assert r["status"] & sbr.STATUS["SBR_RUN"]
    n = g["n_samples"]
    tau_last = g["eta"] * (n - 1) / g["tau_step_den"]
    f = (g["x_first"] - g["x_axis0"]) / (g["x_axis1"] - g["x_axis0"])
    xi_fig = tau_last / (1.0 - f)
    xi_prec = 0.011 / (g["x_axis1"] - g["x_axis0"]) * xi_fig / (1.0 - f)
    assert abs(r["xi"] - xi_fig) <= xi_prec, (r["xi"], xi_fig, xi_prec)
    # the sample count itself: τ_k = 15k/499 ≤ ξ exactly for k < n
    assert int(np.floor(r["xi"] * g["tau_step_den"] / g["eta"])) + 1 == n
    taus = g["eta"] * np.arange(n) / g["tau_step_den"]
    V = np.interp(taus, r["hr_tau"][:len(r["V"])], r["V"])
    assert np.max(np.abs(V - np.array(g["V"]))) <= 2 * g["V_precision"] + 1e-6


def test_interest_hazard_threshold_curves(oracle, golden):
    """hazard_decomposition.pdf: h(τ) and the rV(τ) threshold drawn on one y scale on
    range(0, min(η, ξ), 1000): one fitted scale s (the plot's ylims come from h_f, not
    restated here) must put all 2000 drawn vertices within the 0.01 pt rounding."""
    g = golden("interest_rates.json")["hazard_decomposition"]
    r = _script_point(oracle)
    tau = sbr.julia_range(0.0, min(P["eta"], r["xi"]), 1000)
    h = np.interp(tau, r["hr_tau"], r["hr"])
    rv = P["r"] * np.interp(tau, r["hr_tau"][:len(r["V"])], r["V"])
    yh = np.array(g["y_h"])[::-1] - g["y0"]
    yt = np.array(g["y_rV"])[::-1] - g["y0"]
    # least-squares scale and axis offset over both curves, then every vertex within rounding
    A = np.stack([np.concatenate([rv, h]), np.ones(2 * len(tau))], axis=1)
    (s, off), *_ = np.linalg.lstsq(A, np.concatenate([yt, yh]), rcond=None)
    assert abs(off) < 0.01
    assert np.max(np.abs(yt - (s * rv + off))) <= 0.011
    assert np.max(np.abs(yh - (s * h + off))) <= 0.011


def test_interest_r0_is_the_baseline(oracle):
    """r = 0 takes the baseline branch (interest_rate_solver.jl:95-105): identical results."""
    beta = 1.0 / sbr.julia_range("0.05", "1", 6)
    u = sbr.julia_range("0.001", "0.3", 9)
    a = oracle.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.0, 0.1)
    b = oracle.sweep_baseline(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01)
    for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters"):
        assert np.array_equal(a[k], b[k], equal_nan=a[k].dtype.kind == "f"), k
    assert (a["rk_steps"] == 0).all()


def test_interest_reentry_raises_xi_threshold(oracle):
    """r > 0 adds the option value rV to the threshold (h − rV > u): runs start later
    relative to the baseline at the same u, and the value function starts at (u+δ)/(r+δ)."""
    r = _script_point(oracle)
    assert r["V"][0] == (P["u"] + P["delta"]) / (P["r"] + P["delta"])
    base = oracle.interest_point(P["beta"], P["eta"], P["t_end"], P["u"], P["p"], P["kappa"], P["lam"], 0.0,
                                 P["delta"])
    assert r["tau_in_unc"] > base["tau_in_unc"]
    assert len(r["V"]) == len(r["hr_tau"])


def _grid():
    beta = 1.0 / sbr.julia_range("0.0001", "1", 500)[::50]  # Fig 5 columns (η = 15, tspan (0, 30) carried)
    u = sbr.julia_range("0.001", "1", 500)[::20]
    return beta, u


@pytest.mark.gpu
def test_interest_gpu_bitwise(engine, oracle):
    """GPU interest sweep == the oracle bit for bit (every field, status, bisection count,
    value-function RK step count) on Fig-5 columns at r = 0.06, δ = 0.1, on the script
    point, and the r = 0 branch == the baseline sweep."""
    beta, u = _grid()
    for r, delta, bb, uu in ((0.06, 0.1, beta, u), (0.06, 0.1, [1.0], [0.0, 0.05, 0.1]), (0.02, 0.5, beta[:4], u),
                             (0.0, 0.1, beta, u)):
        g = engine.sweep_interest(bb, 15.0, 30.0, uu, 0.5, 0.6, 0.01, r, delta)
        o = oracle.sweep_interest(bb, 15.0, 30.0, uu, 0.5, 0.6, 0.01, r, delta)
        for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters", "rk_steps"):
            a, b = g[k], o[k]
            same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
            assert same.all(), (r, delta, k, int((~same).sum()))
    g = engine.sweep_interest([1.0], 15.0, 30.0, [0.0], 0.5, 0.6, 0.01, 0.06, 0.1)
    assert g["status"][0, 0] & sbr.STATUS["SBR_RUN"]


def test_interest_capi_argument_errors():
    """The C ABI rejects a null context / result block before any device work (the
    0 <= r < δ check of interest_rate_model.jl:48-50 follows on a live context)."""
    L = sbr.load()
    rc = L.sbr_sweep_interest(None, None, None, None, 1e-4, None, 1, 1, 0.5, 0.6, 0.01, 0.06, 0.1, None, None, None)
    assert rc == sbr._lib.SBR_EARG
    rc = L.sbr_sweep_interest_dev(None, None, None, None, None, 1e-4, None, 1, 1, 0.5, 0.6, 0.01, 0.2, 0.1, None,
                                  None, None)
    assert rc == sbr._lib.SBR_EARG


@pytest.mark.gpu
def test_interest_gpu_rejects_r_not_below_delta(engine):
    with pytest.raises(sbr.ArgumentError):
        engine.sweep_interest([1.0], 15.0, 30.0, [0.1], 0.5, 0.6, 0.01, 0.1, 0.1)


@pytest.mark.gpu
def test_interest_point_paths_bitwise(engine, oracle):
    """sbr_interest_point_paths (the script's single point with its plotted paths: τ̄, HR,
    V saved on the HR grid, AW_cum) == the oracle bit for bit; a no-run u and r = 0 too."""
    for u, r in ((0.0, 0.06), (0.05, 0.06), (0.9, 0.06), (0.1, 0.0)):
        g = engine.interest_point_paths(1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, r, 0.1)
        o = oracle.interest_point(1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, r, 0.1)
        assert g["status"] == o["status"], (u, r)
        for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "hr_tau", "hr", "V", "aw_cum"):
            a, b = np.atleast_1d(g[k]), np.atleast_1d(o[k])
            assert a.shape == b.shape and np.array_equal(a, b, equal_nan=True), (u, r, k)
    assert len(engine.interest_point_paths(1.0, 15.0, 30.0, 0.0, 0.5, 0.6, 0.01, 0.0, 0.1)["V"]) == 0


@pytest.mark.gpu
def test_interest_reference_call_surface(engine, oracle):
    """scripts/3_interest_rates.jl's calls through the host mirror: solve_learning →
    solve_equilibrium_interest → get_AW_functions_interest, equal to the oracle."""
    m = sbr.ModelParametersInterest.make(beta=1.0, eta_bar=15.0, u=0.0, p=0.5, kappa=0.6, lam=0.01, r=0.06,
                                         delta=0.1)
    lr = sbr.solve_learning(m.learning, engine=engine)
    res = sbr.solve_equilibrium_interest(lr, m.economic, m, engine=engine)
    o = _script_point(oracle)
    assert res.xi == o["xi"] and res.bankrun and res.V is not None
    assert np.array_equal(res.V.coefs, o["V"])
    aw = sbr.get_AW_functions_interest(res)
    assert aw["AW_max"] == o["aw_max"]
