"""GPU parity for the social-learning extension: the gfx950 fixed-point
kernels (sbr_social.hip), called through libsbr's C ABI, against the CPU
oracle's restatement of solve_equilibrium_social_learning
(social_learning_solver.jl:63-263) — bit for bit on every output field, every
status bit, the bisection count and the fixed-point iteration count."""
import numpy as np
import pytest

import sbr

pytestmark = pytest.mark.gpu

FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")
ETA = 30.0 / 0.9  # m_social: η = η_bar / β at β = 0.9 (4_social_learning.jl:36-43), carried by copy-modify
P, KAPPA, LAM = 0.99, 0.25, 0.25


def assert_bitwise(a, b, name):
    a = np.asarray(a)
    b = np.asarray(b)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    if not same.all():
        idx = np.argwhere(~same)[:5]
        raise AssertionError(f"{name}: {int((~same).sum())} mismatches, e.g. "
                             f"{[(tuple(i), a[tuple(i)], b[tuple(i)]) for i in idx]}")


def _compare(g, o):
    for k in FIELDS:
        assert_bitwise(g[k], o[k], k)
    assert_bitwise(g["status"], o["status"], "status")
    assert_bitwise(g["iters"], o["iters"], "bisection iterations")
    assert_bitwise(g["fp_iters"], o["fp_iters"], "fixed-point iterations")


def _both(engine, oracle, beta, u, tol=1e-4, max_iter=500):
    cmp = sbr.julia_range(0.0, ETA, 1000)
    g = engine.sweep_social(beta, ETA, u, P, KAPPA, LAM, cmp=cmp, tol=tol, max_iter=max_iter)
    o = oracle.sweep_social(beta, ETA, u, P, KAPPA, LAM, cmp, tol=tol, max_iter=max_iter)
    return g, o


def test_social_script_point(engine, oracle, golden):
    """scripts/4_social_learning.jl:55-56 (β = 0.9, u = 0.5, tol 1e-4, max_iter 500):
    converges (≈50 iterates of ≈10⁵ Tsit5 steps); GPU == oracle, and ξ* matches the figure."""
    g, o = _both(engine, oracle, [0.9], [0.5])
    _compare(g, o)
    gold = golden("social_learning.json")["social"]
    assert g["status"][0, 0] & sbr.STATUS["SBR_RUN"]
    assert not g["status"][0, 0] & sbr.STATUS["SBR_SOCIAL_NOT_CONVERGED"]
    assert abs(g["xi"][0, 0] - gold["xi"]) <= 1.5 * gold["xi_precision"] + 2e-5
    assert g["rk_steps"][0, 0] > 10 ** 6


def test_social_no_run_and_oob_paths(engine, oracle):
    """u above every iterate's hazard (ξ += η/500 branch, converging without a run), and
    two small-u points of the config-5 grid whose fixed point ends in the reference's
    BoundsError (SBR_OOB): one in the bisection's ε lookup past the (0, η) grid, one in
    the forced ODE itself (a stage time past AW_old's last knot → SBR_ODE_FAILED)."""
    g, o = _both(engine, oracle, [0.9], [0.9, 50.0])
    _compare(g, o)
    assert np.all(g["status"] & sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"])
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)
    u = sbr.julia_range("0.001", "1", 512)
    # (found by scanning the oracle over small u: tools/social_oob_scan.py)
    for b, uu, failed in ((beta[40], u[6], False), (beta[0], u[2], True)):
        g, o = _both(engine, oracle, [b], [uu])
        _compare(g, o)
        assert g["status"][0, 0] & sbr.STATUS["SBR_OOB"]
        assert g["status"][0, 0] & sbr.STATUS["SBR_SOCIAL_NOT_CONVERGED"]
        assert bool(g["status"][0, 0] & sbr.STATUS["SBR_ODE_FAILED"]) == failed


def test_social_config5_subgrid_capped(engine, oracle):
    """A subgrid of BASELINE config 5 (β = 1/range(0.01, 2, 512), u = range(0.001, 1, 512))
    with max_iter = 4: every point stops at the cap, so the result is the 4th iterate's
    equilibrium incl. AW_max (social_learning_solver.jl:233-242)."""
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)
    u = sbr.julia_range("0.001", "1", 512)
    bsel = beta[[0, 37, 128, 300, 511]]
    usel = u[[0, 3, 25, 60, 140, 255, 511]]
    g, o = _both(engine, oracle, bsel, usel, max_iter=4)
    _compare(g, o)
    assert (g["fp_iters"] <= 4).all()


def test_social_chunked_workspace(engine):
    """Grids larger than the workspace run in chunks with identical results."""
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)[::40]
    u = sbr.julia_range("0.001", "1", 512)[::40]
    cmp = np.stack([sbr.julia_range(0.0, ETA, 1000)] * len(beta))
    full = engine.sweep_social(beta, ETA, u, P, KAPPA, LAM, cmp=cmp, max_iter=2)
    per_pt = 5 * 98304 * 8 + 1000 * 8 + 64
    small = engine.sweep_social(beta, ETA, u, P, KAPPA, LAM, cmp=cmp, max_iter=2, workspace_bytes=70 * per_pt)
    engine.sweep_social([0.9], ETA, [0.5], P, KAPPA, LAM, cmp=cmp[:1], max_iter=1, workspace_bytes=0)
    assert len(beta) * len(u) > 2 * 70
    for k in FIELDS + ("status", "iters", "fp_iters", "rk_steps"):
        assert_bitwise(small[k], full[k], k)


def test_social_knot_overflow_promotion_and_rerun(engine, oracle):
    """Iterates that outgrow the knot capacity: at 4096 knots points move mid-sweep into
    the 16x pool and redo the iterate from their saved AW_{n-1}; at 1024 knots the pool
    (16384) overflows as well and points re-run from scratch at 65536+.  Every field,
    status bit, iteration count and RK step count equals the default-capacity sweep and
    the oracle."""
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)
    u = sbr.julia_range("0.001", "1", 512)
    bsel = beta[[0, 128, 511]]
    usel = u[[25, 140, 511]]
    cmp = sbr.julia_range(0.0, ETA, 1000)
    o = oracle.sweep_social(bsel, ETA, usel, P, KAPPA, LAM, cmp, max_iter=6)
    ref = engine.sweep_social(bsel, ETA, usel, P, KAPPA, LAM, cmp=cmp, max_iter=6)
    assert engine.social_overflow_stats() == dict(promoted=0, rerun=0)
    _compare(ref, o)
    for cap, want in ((4096, "promoted"), (1024, "rerun")):
        g = engine.sweep_social(bsel, ETA, usel, P, KAPPA, LAM, cmp=cmp, max_iter=6, knot_capacity=cap)
        stats = engine.social_overflow_stats()
        assert stats[want] > 0, (cap, stats)
        _compare(g, o)
        assert_bitwise(g["rk_steps"], ref["rk_steps"], f"rk_steps at capacity {cap}")
        assert not (g["status"] & sbr.STATUS["SBR_KNOT_OVERFLOW"]).any()


def test_social_promoted_points_reach_max_iter(engine, oracle):
    """Points that never converge (tol = 1e-300) and outgrow an 8192-knot capacity: they are
    promoted into the pool during the first launches and trail the main worklist by up to one
    launch's iterates, so the pool must be drained past the main list's last launch until
    every promoted point has run all max_iter = 30 iterates (one 8-iterate drain
    left such points live, their results unwritten).  GPU == oracle on every field."""
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)
    u = sbr.julia_range("0.001", "1", 512)
    bsel, usel = beta[[128, 511]], u[[140, 25]]
    cmp = sbr.julia_range(0.0, ETA, 1000)
    o = oracle.sweep_social(bsel, ETA, usel, P, KAPPA, LAM, cmp, tol=1e-300, max_iter=30)
    g = engine.sweep_social(bsel, ETA, usel, P, KAPPA, LAM, cmp=cmp, tol=1e-300, max_iter=30, knot_capacity=8192)
    stats = engine.social_overflow_stats()
    assert stats["promoted"] > 0 and stats["rerun"] == 0, stats
    _compare(g, o)
    assert (g["fp_iters"] == 30).all()
    assert (g["status"] & sbr.STATUS["SBR_SOCIAL_NOT_CONVERGED"]).all()


def test_social_point_paths_bitwise(engine, oracle):
    """sbr_social_point_paths: the returned SolvedModel's learning knots (t, G) — from which
    scripts/4_social_learning.jl's AW curves are rebuilt — equal the oracle's, on the script
    point and on a BoundsError point (where the previous iterate's SolvedModel is returned)."""
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)
    u = sbr.julia_range("0.001", "1", 512)
    cmp = sbr.julia_range(0.0, ETA, 1000)
    for b, uu in ((0.9, 0.5), (beta[40], u[6])):
        g = engine.social_point_paths(b, ETA, uu, P, KAPPA, LAM, cmp=cmp)
        o = oracle.social_point(b, ETA, uu, P, KAPPA, LAM, cmp)
        assert g["status"] == o["status"] and g["fp_iters"] == o["fp_iters"], (b, uu)
        for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "t", "G", "aw_old"):
            x, y = np.atleast_1d(g[k]), np.atleast_1d(o[k])
            assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), (b, uu, k)


@pytest.mark.parametrize("fixture", ["config5_sample.npz", "config5_sample_1024.npz"])
def test_social_config5_sample_full_workload(engine, golden, fixture):
    """BASELINE config 5 at its stated workload (tol 1e-4, max_iter 500) on an 8 β × 4 u
    sample of the 512² axes, incl. the corner β = 100, u = 0.001, and on the stratified
    1,024-point sample (every 16th β × every 16th u, corner included): bit for bit against
    the oracle's fixed points (tests/golden/config5_sample*.npz, tools/make_config5_sample.py
    [--stride 16]) on every field, status bit, bisection and fixed-point iteration count."""
    gold = golden(fixture)
    cmp = np.stack([sbr.julia_range(0.0, ETA, 1000)] * len(gold["beta"]))
    g = engine.sweep_social(gold["beta"], ETA, gold["u"], P, KAPPA, LAM, cmp=cmp, tol=1e-4, max_iter=500)
    for k in FIELDS:
        assert_bitwise(g[k], gold[k], k)
    assert_bitwise(g["status"], gold["status"], "status")
    assert_bitwise(g["iters"], gold["iters"], "bisection iterations")
    assert_bitwise(g["fp_iters"], gold["fp_iters"], "fixed-point iterations")
    assert (g["status"] & sbr.STATUS["SBR_RUN"]).any() and (g["status"] & sbr.STATUS["SBR_OOB"]).any()


def test_social_point_engine_hr_and_aw_paths(engine, oracle):
    """The social drop-in's HR and get_AW paths come from the engine (SBRDropInSocial.jl):
    sbr_equilibrium_on_knots_pdf on the returned knots with pdf = ((1 − G)·β)·AW_{n−1}
    (compute_pdf_social_learning, social_learning_dynamics.jl:98-114) reproduces the social
    point's last inner equilibrium bit for bit, and its τ̄ / HR / AW_cum / AW_OUT / AW_IN equal
    the oracle's hazard_rate + get_AW on the same pdf — on a run and on a no-run point."""
    for b, uu in ((0.9, 0.5), (0.9, 50.0)):
        g = engine.social_point_paths(b, ETA, uu, P, KAPPA, LAM)
        pdf = ((1.0 - g["G"]) * b) * g["aw_old"]
        e = engine.equilibrium_on_knots(g["t"], g["G"], b, ETA, ETA, uu, P, KAPPA, LAM, pdf=pdf)
        for k in FIELDS:
            assert np.array_equal(e[k][0], g[k], equal_nan=True), (b, uu, k, e[k][0], g[k])
        run = sbr.STATUS["SBR_RUN"]
        assert (int(e["status"][0]) & run) == (g["status"] & run)
        o = oracle.equilibrium_paths_pdf(g["t"], g["G"], pdf, ETA, ETA, uu, P, KAPPA, LAM)
        assert o["status"] == int(e["status"][0])
        for k in ("hr_tau", "hr", "aw_cum", "aw_out", "aw_in"):
            x = e["tau" if k == "hr_tau" else k]
            assert x.shape == o[k].shape and np.array_equal(x, o[k], equal_nan=True), (b, uu, k)


def test_social_config5_strided_points_full_workload(engine, oracle):
    """BASELINE config 5 at its stated workload (tol 1e-4, max_iter 500) on 128 points of the
    512² axes — every 64th β × every 32nd u, a stratified sample four times the golden
    fixture's — bit for bit against the oracle's fixed points computed here (every field,
    status bit, bisection and fixed-point iteration count)."""
    beta = (1.0 / sbr.julia_range("0.01", "2", 512))[::64]
    u = sbr.julia_range("0.001", "1", 512)[::32]
    g, o = _both(engine, oracle, beta, u, tol=1e-4, max_iter=500)
    _compare(g, o)
    st = g["status"]
    assert (st & sbr.STATUS["SBR_RUN"]).any() and ((st & sbr.STATUS["SBR_RUN"]) == 0).any()
