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


def test_workspace_growth_between_single_and_vector_calls(oracle):
    """A fresh context: one-u calls (mapped-memory path), then a u vector past the workspace's
    initial capacity (it is reallocated, mapped block included), then one-u calls again —
    every result equal to the oracle (the reallocation leaves no stale error or buffer)."""
    eng = sbr.Engine(0)
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    P = dict(beta=1.0, eta=15.0, t_end=30.0, p=0.5, kappa=0.6, lam=0.01)
    us = sbr.julia_range("0.001", "0.2", 5000)[:2700]
    for u in (float(us[5]), float(us[2000])):
        g, o = solve_both(eng, oracle, t, G, P, u=u)
        check_point(g, o, f"single {u}")
    g = eng.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, us, 0.5, 0.6, 0.01, paths=False)
    for j in range(0, 2700, 271):
        o = oracle.equilibrium(t, G, 1.0, 15.0, 30.0, float(us[j]), 0.5, 0.6, 0.01)
        for f in FIELDS:
            assert same(g[f][j], o[f]), (j, f)
        assert int(g["status"][j]) == o["status"] and int(g["iters"][j]) == o["iters"], j
    for u in (float(us[7]), float(us[2699])):
        g, o = solve_both(eng, oracle, t, G, P, u=u)
        check_point(g, o, f"single again {u}")


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


# ---------------------------------------------------------------- heterogeneity extension
HFIELDS = ("xi", "aw_max", "tol")


def check_hetero(g, o, name, paths=True):
    for f in HFIELDS:
        assert same(g[f], o[f]), (name, f, g[f], o[f])
    assert np.array_equal(g["status"], o["status"]), (name, g["status"], o["status"])
    assert np.array_equal(g["iters"], o["iters"]), name
    for f in ("tau_in_unc", "tau_out_unc"):
        assert same(g[f], o[f]), (name, f)
    if paths:
        assert g["n_tau"] == o["n_hr"], name
        assert same(g["hr"], o["hr"]), (name, "hr")
        if o["status"][0] & sbr.STATUS["SBR_RUN"]:
            assert same(g["aw_total"], o["aw_total"]), (name, "aw_total")


def test_hetero_on_caller_knots_bitwise(engine, oracle):
    """sbr_hetero_equilibrium_on_knots on the script column's learning knots (the oracle's
    solve_SInetwork_hetero): every field, the per-group buffers, HR_k on the τ̄ grid (the
    SolvedModelHetero.HRs, heterogeneity_solver.jl:255) and AW_total equal the oracle on the
    same knots; the point equals sbr_hetero_point_paths (which learns); perturbed group CDFs
    give the perturbed knots' equilibrium."""
    g = sbr.hetero_script_grid()
    betas, dist = g.betas[0], g.dist
    t, G, _ = oracle.learn_hetero(betas, dist, g.t_end[0])
    for u in (float(g.u[0]), 0.9):
        a = engine.hetero_equilibrium_on_knots(t, G, betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
        o = oracle.hetero_equilibrium_knots(t, G, betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
        check_hetero(a, o, f"u={u}")
        pp = engine.hetero_point_paths(betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
        assert same(a["xi"][0], pp["xi"]) and same(a["aw_max"][0], pp["aw_max"])
        if a["status"][0] & sbr.STATUS["SBR_RUN"]:
            assert np.array_equal(a["aw_total"], pp["aw_total"])
    u = float(g.u[0])
    Gp = np.ascontiguousarray(G * (1 - 1e-9))
    a = engine.hetero_equilibrium_on_knots(t, Gp, betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
    o = oracle.hetero_equilibrium_knots(t, Gp, betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
    check_hetero(a, o, "perturbed")
    b = engine.hetero_equilibrium_on_knots(t, G, betas, dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
    assert a["xi"][0] != b["xi"][0] or a["aw_max"][0] != b["aw_max"][0]


def test_hetero_config4_column_u_vector(engine, oracle):
    """A config-4 column (K = 8, Rosenbrock23 knots) with 40 u values in one call, and its
    η past the knots (the hazard's BoundsError)."""
    c4 = sbr.hetero_config4(64, 40, 8)
    i = 37
    t, G, _ = oracle.learn_hetero(c4.betas[i], c4.dist, c4.t_end[i])
    a = engine.hetero_equilibrium_on_knots(t, G, c4.betas[i], c4.dist, c4.eta[i], c4.t_end[i], c4.u, c4.p, c4.kappa,
                                           c4.lam, paths=False)
    o = oracle.hetero_equilibrium_knots(t, G, c4.betas[i], c4.dist, c4.eta[i], c4.t_end[i], c4.u, c4.p, c4.kappa,
                                        c4.lam)
    check_hetero(a, o, "config4", paths=False)
    assert (a["status"] & sbr.STATUS["SBR_RUN"]).any()
    a = engine.hetero_equilibrium_on_knots(t, G, c4.betas[i], c4.dist, 2 * float(t[-1]), c4.t_end[i], 0.1, c4.p,
                                           c4.kappa, c4.lam)
    o = oracle.hetero_equilibrium_knots(t, G, c4.betas[i], c4.dist, 2 * float(t[-1]), c4.t_end[i], 0.1, c4.p,
                                        c4.kappa, c4.lam)
    check_hetero(a, o, "eta_past_knots")
    assert a["status"][0] & sbr.STATUS["SBR_OOB"] and a["n_tau"] == 0


def test_hetero_mirror_learns_once(engine, oracle):
    """scripts/2_heterogeneity.jl through the mirror: solve_SInetwork_hetero once, then
    solve_equilibrium_hetero(lr, econ) per u on lr's knots; HRs are the engine's HR_k."""
    g = sbr.hetero_script_grid()
    m = sbr.ModelParametersHetero.make(g.betas[0], g.dist, eta_bar=30.0, u=float(g.u[0]), p=g.p, kappa=g.kappa,
                                       lam=g.lam)
    lr = sbr.solve_SInetwork_hetero(m.learning, engine)
    t, G, _ = oracle.learn_hetero(g.betas[0], g.dist, m.learning.tspan[1])
    assert np.array_equal(lr.grid, t) and np.array_equal(lr.G, G)
    for u in (float(g.u[0]), 0.5):
        e = sbr.ModelParametersHetero.modify(m, u=u).economic
        r = sbr.solve_equilibrium_hetero(lr, e, engine=engine)
        o = oracle.hetero_equilibrium_knots(t, G, g.betas[0], g.dist, e.eta, m.learning.tspan[1], u, g.p, g.kappa,
                                            g.lam)
        assert r.xi == o["xi"][0] or (np.isnan(r.xi) and np.isnan(o["xi"][0]))
        assert len(r.HRs) == len(g.dist)
        for k, hr in enumerate(r.HRs):
            assert np.array_equal(hr.coefs, o["hr"][k])


# ------------------------------------------------ AW_max bounds at the knot-separation edges
def _crowd(t, G, picks, sep, K=None):
    """t / G with one extra knot after each index in `picks`, `sep`·t[n−1] past it (G between its
    neighbours' values, so G stays nondecreasing): consecutive knots just above (sep = 2e-15) or
    below (sep = 0.5e-15) the 1e-15·t[n−1] separation the AW bounds test (Summ::koff)."""
    tn, Gn = [t[0]], [G[0]]
    for i in range(len(t) - 1):
        if i in picks:
            tn.append(t[i] + sep * t[-1])
            Gn.append(G[i] + (G[i + 1] - G[i]) * 1e-3)
        tn.append(t[i + 1])
        Gn.append(G[i + 1])
    return np.asarray(tn), np.asarray(Gn) if K is None else np.stack(Gn)


@pytest.mark.parametrize("sep", [2e-15, 0.5e-15])
def test_aw_bounds_at_knot_separation_edge(engine, oracle, sep):
    """AW_OUT(b_j) is bounded by G[j + 1] only when consecutive knots are more than
    1e-15·t[n−1] apart (else G[j + 2]), and by G[j] where b_j = t[j] exactly (SBR_AW_OWN).  Knots
    crowded to 2e-15 / 0.5e-15·t[n−1] around the AW peak, the buffers and ξ of a u sweep: the
    pruned AW_max (aw_scan / branch and bound) equals the exhaustive evaluation bit for bit,
    and both equal the oracle."""
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    picks = set(range(200, len(t) - 200, 37))
    tc, Gc = _crowd(t, G, picks, sep)
    assert np.all(np.diff(tc) > 0) and np.all(np.diff(Gc) >= 0)
    u = sbr.julia_range("0.001", "0.2", 400)
    a = engine.equilibrium_on_knots(tc, Gc, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, paths=False)
    b = engine.equilibrium_on_knots(tc, Gc, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, paths=False, exhaustive=True)
    for f in FIELDS:
        assert same(a[f], b[f]), f
    assert np.array_equal(a["status"], b["status"]) and np.array_equal(a["iters"], b["iters"])
    run = (a["status"] & sbr.STATUS["SBR_RUN"]) > 0
    assert run.sum() > 100
    for j in range(0, 400, 23):
        o = oracle.equilibrium(tc, Gc, 1.0, 15.0, 30.0, float(u[j]), 0.5, 0.6, 0.01)
        for f in FIELDS:
            assert same(a[f][j], o[f]), (j, f)


@pytest.mark.parametrize("sep", [2e-15, 0.5e-15])
def test_hetero_aw_bounds_at_knot_separation_edge(engine, oracle, sep):
    """The same for the heterogeneity branch and bound (SBR_HET_K1): a config-4 column's knots
    crowded to 2e-15 / 0.5e-15·t[n−1], 60 u: pruned == exhaustive bit for bit."""
    c4 = sbr.hetero_config4(64, 60, 8)
    i = 37
    t, G, _ = oracle.learn_hetero(c4.betas[i], c4.dist, c4.t_end[i])
    picks = set(range(100, len(t) - 100, 29))
    tc, Gc = _crowd(t, list(G), picks, sep, K=8)
    assert np.all(np.diff(tc) > 0)
    args = (tc, np.ascontiguousarray(Gc), c4.betas[i], c4.dist, c4.eta[i], c4.t_end[i], c4.u, c4.p, c4.kappa, c4.lam)
    a = engine.hetero_equilibrium_on_knots(*args, paths=False)
    b = engine.hetero_equilibrium_on_knots(*args, paths=False, exhaustive=True)
    check_hetero(a, b, "pruned vs exhaustive", paths=False)
    assert (a["status"] & sbr.STATUS["SBR_RUN"]).any()


def test_knots_pdf_matches_oracle(engine, oracle):
    """sbr_equilibrium_on_knots_pdf: an explicit pdf on the knots (here βG(1 − G)·(1 + G) and
    the pdf βG(1 − G) itself) — single point with paths, a u vector, η at the knots' edges —
    bitwise equal to the oracle's hazard_rate + equilibrium on the same pdf; alternating with
    the symbolic-pdf call on the same knots swaps the resident hazard (cache keyed by pdf)."""
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    P = dict(eta=15.0, t_end=30.0, p=0.5, kappa=0.6, lam=0.01)
    sym = (1.0 * G) * (1.0 - G)
    shaped = sym * (1.0 + G)
    for rep in range(2):
        for name, pdf in (("shaped", shaped), ("symbolic", sym)):
            for u in (0.02, 0.3, 5.0):
                g = engine.equilibrium_on_knots(t, G, 7.0, P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"],
                                                pdf=pdf)
                o = oracle.equilibrium_paths_pdf(t, G, pdf, P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"])
                check_point(g, o, f"{name} {u} {rep}")
            s = engine.equilibrium_on_knots(t, G, 1.0, P["eta"], P["t_end"], 0.3, P["p"], P["kappa"], P["lam"])
            o = oracle.equilibrium_paths(t, G, 1.0, P["eta"], P["t_end"], 0.3, P["p"], P["kappa"], P["lam"])
            check_point(s, o, f"plain after {name}")
    # the explicit βG(1 − G) is the symbolic path
    a = engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, 0.3, 0.5, 0.6, 0.01)
    b = engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, 0.3, 0.5, 0.6, 0.01, pdf=sym)
    for k in FIELDS + ("tau", "hr", "aw_cum", "aw_out", "aw_in"):
        assert same(a[k], b[k]), k
    u = sbr.julia_range("0.0", "1.2", 301)
    g = engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01, paths=False, pdf=shaped)
    for j in range(0, 301, 20):
        o = oracle.equilibrium_paths_pdf(t, G, shaped, 15.0, 30.0, float(u[j]), 0.5, 0.6, 0.01)
        for f in FIELDS:
            assert same(g[f][j], o[f]), (j, f)
        assert int(g["status"][j]) == o["status"] and int(g["iters"][j]) == o["iters"], j
    for eta in (float(t[-1]), 45.0):
        g = engine.equilibrium_on_knots(t, G, 1.0, eta, 30.0, 0.1, 0.5, 0.6, 0.01, pdf=shaped)
        o = oracle.equilibrium_paths_pdf(t, G, shaped, eta, 30.0, 0.1, 0.5, 0.6, 0.01)
        for f in FIELDS:
            assert same(g[f][0], o[f]), (eta, f)
        assert int(g["status"][0]) == o["status"] and len(g["tau"]) == o["n_hr"], eta
    with pytest.raises(sbr.ArgumentError):
        engine.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, 0.1, 0.5, 0.6, 0.01, pdf=shaped[:-1])
