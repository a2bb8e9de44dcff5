"""Social-learning extension (src/extensions/social_learning/*.jl).

CPU: the oracle's restatement of solve_equilibrium_social_learning
(social_learning_solver.jl:63-263) pinned to the reference's committed figure
output/figures/social_learning/social_learning_equilibrium.pdf
(scripts/4_social_learning.jl:55-56, 104-106; tests/golden/social_learning.json).
"""
import numpy as np
import pytest

import sbr
from golden_util import aw_paths, interp


def _social_case(golden):
    g = golden("social_learning.json")["social"]
    P = g["params"]
    eta = P["eta_bar"] / P["beta"]  # ModelParameters kw ctor: η = η_bar / β (model.jl:162-164)
    cmp = sbr.julia_range(0.0, eta, 1000)  # social_learning_solver.jl:103
    return g, P, eta, cmp


def test_comparison_grid_is_julia_range():
    eta = 30.0 / 0.9
    cmp = sbr.julia_range(0.0, eta, 1000)
    assert cmp[0] == 0.0 and cmp[-1] == eta  # range endpoints are exact
    assert np.all(np.diff(cmp) > 0)
    # Base.rat finds 100/3 for η, so element k is the rounded k·(100/3)/999
    from fractions import Fraction
    assert all(cmp[k] == float(Fraction(100, 3) * k / 999) for k in (1, 7, 500, 998))


def test_social_script_figure(oracle, golden):
    """ξ*, τ_IN and the plotted AW_cum/AW_OUT/AW_IN of the last iterate (plot_equilibrium
    on the returned SolvedModel, plotting.jl:156-210) against the figure."""
    g, P, eta, cmp = _social_case(golden)
    r = oracle.social_point(P["beta"], eta, P["u"], P["p"], P["kappa"], P["lam"], cmp, tol=P["tol"],
                            max_iter=P["max_iter"])
    assert r["status"] & sbr.STATUS["SBR_RUN"]
    assert not r["status"] & sbr.STATUS["SBR_SOCIAL_NOT_CONVERGED"]
    assert r["t"][-1] == eta  # tspan overridden to (0, η) (social_learning_solver.jl:79)
    xi = r["xi"]
    assert abs(xi - g["xi"]) <= 1.5 * g["xi_precision"] + 2e-5
    assert abs((xi - r["tau_in_unc"]) - g["tau_in"]) <= 1.5 * g["tau_in_precision"] + 2e-5
    n = g["n_samples"]
    ts = np.arange(n) / 10.0
    cum, out, inn = aw_paths(xi, r["tau_in_unc"], r["tau_out_unc"], r["hr_tau"], r["t"], r["G"])
    tol_y = 1.5 * g["aw_precision"] + 1e-5
    for name, path in (("aw_cum", cum), ("aw_out", out), ("aw_in", inn)):
        got = interp(r["hr_tau"], path, ts)
        assert np.max(np.abs(got - np.array(g[name]))) <= tol_y, name
    assert abs(r["aw_max"] - np.max(cum)) == 0.0
    # social learning delays the run relative to word of mouth (Δξ = ξ_social − ξ_baseline < 0 here)
    gb = golden("social_learning.json")["baseline"]
    assert xi < gb["xi"]


def test_social_sweep_matches_point(oracle, golden):
    """The sweep entry point gives the single-point result bit for bit."""
    g, P, eta, cmp = _social_case(golden)
    r = oracle.social_point(P["beta"], eta, P["u"], P["p"], P["kappa"], P["lam"], cmp, tol=P["tol"],
                            max_iter=P["max_iter"])
    s = oracle.sweep_social([P["beta"]], eta, [P["u"]], P["p"], P["kappa"], P["lam"], cmp, tol=P["tol"],
                            max_iter=P["max_iter"])
    for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol"):
        assert s[k][0, 0] == r[k] or (np.isnan(s[k][0, 0]) and np.isnan(r[k])), k
    assert s["status"][0, 0] == r["status"]
    assert s["fp_iters"][0, 0] == r["fp_iters"]


def test_social_no_run_branch(oracle):
    """u above max HR in every iterate: the ξ += η/500 branch (social_learning_solver.jl:150-156)
    runs until ξ > η (:152-156) or the undamped AW stops moving (:165-172)."""
    eta = 30.0 / 0.9
    cmp = sbr.julia_range(0.0, eta, 1000)
    s = oracle.sweep_social([0.9], eta, [50.0], 0.99, 0.25, 0.25, cmp, tol=1e-4, max_iter=500)
    st = int(s["status"][0, 0])
    assert not st & sbr.STATUS["SBR_RUN"]
    assert np.isnan(s["xi"][0, 0]) and np.isinf(s["tol"][0, 0]) or s["tol"][0, 0] == 0.0
    assert st & sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"]
