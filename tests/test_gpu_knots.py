"""GPU parity of sbr_equilibrium_on_knots — solve_equilibrium_baseline(lr, econ) +
get_AW_functions! (solver.jl:413-462, 495-576) on the learning knots the caller holds, with
no learning ODE — against the oracle's restatement on the same knots (sbro_equilibrium_paths),
bit for bit: every result field, the status bits, the bisection count, the hazard grid and
HR, and get_AW's AW_cum / AW_OUT / AW_IN paths.  Perturbed knots prove the caller's
LearningResults is what is solved; the resident-knot cache is checked across calls."""
import numpy as np
import pytest

import sbr

pytestmark = pytest.mark.gpu

FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))


def check_point(g, o, name):
    for f in FIELDS:
        assert same(g[f][0], o[f]), (name, f, g[f][0], o[f])
    assert int(g["status"][0]) == o["status"], (name, hex(int(g["status"][0])), hex(o["status"]))
    assert int(g["iters"][0]) == o["iters"], name
    assert same(g["tau"], o["hr_tau"]), (name, "tau")
    assert same(g["hr"], o["hr"]), (name, "hr")
    if o["status"] & sbr.STATUS["SBR_RUN"]:
        for k in ("aw_cum", "aw_out", "aw_in"):
            assert same(g[k], o[k]), (name, k)
    else:
        assert np.isnan(g["aw_cum"]).all()


def solve_both(engine, oracle, t, G, P, u=None):
    u = P["u"] if u is None else u
    g = engine.equilibrium_on_knots(t, G, P["beta"], P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"])
    o = oracle.equilibrium_paths(t, G, P["beta"], P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"])
    return g, o


@pytest.mark.parametrize("case", ["main", "fast", "low_u"])
def test_fig3_on_caller_knots_bitwise(engine, oracle, golden, case):
    """The Fig 3 equilibria on the oracle's own learning knots (what a LearningResults
    holds): bit-identical to the oracle, and ξ on the figure."""
    P = golden("fig3_equilibria.json")[case]["params"]
    t, G, _ = oracle.learn_logistic(P["beta"], P["t_end"])
    g, o = solve_both(engine, oracle, t, G, P)
    check_point(g, o, case)
    gx = golden("fig3_equilibria.json")[case]
    assert abs(g["xi"][0] - gx["xi"]) <= 1.5 * gx["xi_precision"] + 2e-5


def test_perturbed_knots_are_the_ones_solved(engine, oracle, golden):
    """A caller who hands other knots gets the equilibrium of those knots: G scaled by
    (1 + 1e-7), the grid refined by midpoints (2n − 1 knots: past the LDS slab, the
    global-memory kernel), a shifted time axis — each bit-identical to the oracle on the
    same knots and different from the unperturbed solve; then the original knots again
    (the resident copy is replaced and restored by value)."""
    P = golden("fig3_equilibria.json")["main"]["params"]
    t, G, _ = oracle.learn_logistic(P["beta"], P["t_end"])
    g0, o0 = solve_both(engine, oracle, t, G, P)
    check_point(g0, o0, "base")
    tm = np.empty(2 * len(t) - 1)
    tm[0::2], tm[1::2] = t, 0.5 * (t[:-1] + t[1:])
    Gm = np.empty_like(tm)
    Gm[0::2], Gm[1::2] = G, 0.5 * (G[:-1] + G[1:])
    info = engine.device_info()
    assert len(tm) > info["lds_knot_capacity"] // 2 or len(tm) > 4432  # sized past the baseline slab
    variants = {"scaled_G": (t, G * (1 + 1e-7)), "refined": (tm, Gm), "shifted_t": (t * (1 + 1e-9), G)}
    for name, (tv, Gv) in variants.items():
        g, o = solve_both(engine, oracle, tv, Gv, P)
        check_point(g, o, name)
        assert g["xi"][0] != g0["xi"][0] or g["aw_max"][0] != g0["aw_max"][0], name
    g1, _ = solve_both(engine, oracle, t, G, P)
    check_point(g1, o0, "restored")


def test_u_vector_and_resident_cache(engine, oracle):
    """n_u = 777 points of one LearningResults in one call, and the same u one per call
    (knots and HR resident after the first): identical, and equal to the oracle per point
    (no-run, run and u above every HR value included)."""
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    u = sbr.julia_range("0.0", "1.2", 777)
    P = dict(beta=1.0, eta=15.0, t_end=30.0, p=0.5, kappa=0.6, lam=0.01)
    g = engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, paths=False)
    for j in range(0, 777, 7):
        o = oracle.equilibrium(t, G, 1.0, 15.0, 30.0, float(u[j]), 0.5, 0.6, 0.01)
        for f in FIELDS:
            assert same(g[f][j], o[f]), (j, f)
        assert int(g["status"][j]) == o["status"] and int(g["iters"][j]) == o["iters"], j
        if j % 49 == 0:
            one = engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, float(u[j]), 0.5, 0.6, 0.01)
            for f in FIELDS:
                assert same(one[f][0], g[f][j]), (j, f)
    run = (g["status"] & sbr.STATUS["SBR_RUN"]) > 0
    assert run.any() and (~run).any()
    # a different η / p / λ with the same knots recomputes the hazard (cache key)
    for kw in (dict(eta=12.0), dict(p=0.7), dict(lam=0.02)):
        Q = {**P, **kw, "u": 0.05}
        a, b = solve_both(engine, oracle, t, G, Q)
        check_point(a, b, str(kw))


@pytest.mark.parametrize("case", ["eta_past_knots", "eta_is_last_knot", "eta_before_first"])
def test_hazard_edges(engine, oracle, case):
    """η past the last knot (pdf(η) is the interpolant's BoundsError), η equal to the last
    knot (not appended), and knots starting after η: status and paths as the oracle's."""
    t, G, _ = oracle.learn_logistic(2.0, 20.0)
    P = dict(beta=2.0, t_end=20.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
    if case == "eta_past_knots":
        P["eta"] = 25.0
    elif case == "eta_is_last_knot":
        P["eta"] = float(t[-1])
    else:
        t = t + 3.0
        P["eta"] = 2.0
    g, o = solve_both(engine, oracle, t, G, P)
    for f in FIELDS:
        assert same(g[f][0], o[f]), (case, f)
    assert int(g["status"][0]) == o["status"], case
    assert len(g["tau"]) == o["n_hr"]
    if case != "eta_is_last_knot":
        assert o["status"] & sbr.STATUS["SBR_OOB"]
        assert len(g["tau"]) == 0


def test_unsorted_knots_are_an_argument_error(engine, oracle):
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    t2 = t.copy()
    t2[10], t2[11] = t2[11], t2[10]
    with pytest.raises(sbr.ArgumentError):
        engine.equilibrium_on_knots(t2, G, 1.0, 15.0, 30.0, 0.1, 0.5, 0.6, 0.01)
    with pytest.raises(sbr.ArgumentError):
        engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, [0.1, 0.2], 0.5, 0.6, 0.01, paths=True)


def test_unchanged_fig4_loop_equals_batched_sweep(engine):
    """scripts/1_baseline.jl's Fig 4 loop run unchanged through the Python mirror — one
    solve_learning, then solve_equilibrium_baseline + get_AW_functions per u with the 5-NaN
    early termination (:151-192) — gives bit for bit the batched sweep's Fig 4 column
    (sbr_sweep_baseline with early_exit = 5), and the figure's 2,718 run points."""
    m = sbr.ModelParameters.make(beta=1.0, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
    lr = sbr.solve_learning(m.learning, engine)
    grid = sbr.fig4_grid(5000)
    ref = engine.sweep_baseline(grid, early_exit=5)
    aw, xi, ret = [], [], []
    nan_run = 0
    for u in grid.u:
        if nan_run >= 5:
            break
        m_u = sbr.ModelParameters.modify(m, u=float(u))  # ModelParameters(m_base; u=u), :168
        r = sbr.solve_equilibrium_baseline(lr, m_u.economic, engine)
        a = sbr.get_AW_functions(r)
        if r.bankrun:
            aw.append(a["AW_max"]); xi.append(r.xi); ret.append(r.xi - r.tau_bar_IN_UNC)
            nan_run = 0
        else:
            aw.append(np.nan); xi.append(np.nan); ret.append(np.nan)
            nan_run += 1
    k = len(aw)
    assert same(np.array(aw), ref["aw_max"][0, :k])
    assert same(np.array(xi), ref["xi"][0, :k])
    assert np.isnan(ref["aw_max"][0, k:]).all()
    assert int(np.isfinite(aw).sum()) == 2718
