"""compute_ξ's ξ_guess (solver.jl:309-312; solve_equilibrium_baseline(lr, econ; ξ_guess) passes it
through, :413,441): the bisection's first iterate.  The oracle restates it (sbro_set_xi_guess); the
engine honours it on the caller's knots (sbr_equilibrium_on_knots, opts.xi_guess) with the
reference's plain iteration and refuses it on the sweeps.  GPU == oracle bit for bit for guesses
inside the buffers, outside them, off the knot grid (the interpolant's BoundsError) and at the
midpoint (== the default, iteration count included)."""
import ctypes

import numpy as np
import pytest

import sbr
from sbr import _lib

FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")
P = dict(beta=1.0, eta=15.0, t_end=30.0, p=0.5, kappa=0.6, lam=0.01)


def _same(a, b):
    return (a == b) or (np.isnan(a) and np.isnan(b))


def _oracle(oracle, t, G, u, guess):
    oracle.set_xi_guess(guess)
    try:
        return oracle.equilibrium(t, G, P["beta"], P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"])
    finally:
        oracle.set_xi_guess()


def test_oracle_guess_at_midpoint_is_the_default(oracle):
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    d = _oracle(oracle, t, G, 0.1, float("nan"))
    m = _oracle(oracle, t, G, 0.1, (d["tau_in_unc"] + d["tau_out_unc"]) / 2.0)
    for f in FIELDS:
        assert _same(d[f], m[f]), f
    assert d["status"] == m["status"] and d["iters"] == m["iters"]
    g = _oracle(oracle, t, G, 0.1, d["xi"] + 0.3)  # another first iterate: another path, same root region
    assert g["status"] & sbr.STATUS["SBR_RUN"] and g["iters"] != d["iters"]
    assert abs(g["xi"] - d["xi"]) < 1e-9
    assert _oracle(oracle, t, G, 0.1, -1.0)["status"] & sbr.STATUS["SBR_OOB"]  # ξ_old below the grid


@pytest.mark.gpu
def test_guess_gpu_equals_oracle(engine, oracle):
    t, G, _ = oracle.learn_logistic(1.0, 30.0)
    us = [0.01, 0.1, 0.105, 0.2]
    for u in us:
        d = _oracle(oracle, t, G, u, float("nan"))
        tin, tout = d["tau_in_unc"], d["tau_out_unc"]
        guesses = [float("nan"), (tin + tout) / 2.0, tin + 0.1, tout - 0.1, tout + 1.0, tin - 0.5, 0.0, -1.0,
                   29.9999, 31.0, 1e300]
        for g in guesses:
            o = _oracle(oracle, t, G, u, g)
            for paths in (True, False):  # the single-point kernel, the u-vector kernel
                uu = u if paths else np.array([u, u])
                r = engine.equilibrium_on_knots(t, G, P["beta"], P["eta"], P["t_end"], uu, P["p"], P["kappa"],
                                                P["lam"], paths=paths, xi_guess=None if g != g else g)
                for k in range(1 if paths else 2):
                    for f in FIELDS:
                        assert _same(r[f][k], o[f]), (u, g, paths, f, r[f][k], o[f])
                    assert int(r["status"][k]) == o["status"], (u, g, paths, hex(int(r["status"][k])), hex(o["status"]))
                    assert int(r["iters"][k]) == o["iters"], (u, g, paths)
        # the midpoint guess takes the plain iteration and lands on the default's bits, count included
        dm = engine.equilibrium_on_knots(t, G, P["beta"], P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"])
        gm = engine.equilibrium_on_knots(t, G, P["beta"], P["eta"], P["t_end"], u, P["p"], P["kappa"], P["lam"],
                                         xi_guess=(tin + tout) / 2.0)
        for f in FIELDS + ("status", "iters"):
            assert _same(float(dm[f][0]), float(gm[f][0])), (u, f)


@pytest.mark.gpu
def test_sweeps_refuse_a_guess(engine):
    L = _lib.load()
    g = sbr.fig5_grid(8, n_u=4)
    nb, nu = len(g.beta), len(g.u)
    out = {k: np.empty(nb * nu) for k in FIELDS}
    out["status"] = np.empty(nb * nu, np.uint32)
    soa = _lib.ResultSoA(*[out[k].ctypes.data_as(ctypes.c_void_p) for k in (*FIELDS, "status")], None)
    opts = _lib.default_opts(xi_guess=5.0, flags=_lib.SBR_FLAG_XI_GUESS)
    P_ = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = L.sbr_sweep_baseline(engine._ctx, P_(g.beta), P_(g.eta), P_(g.t_end), g.x0, P_(g.u), nb, nu, g.p, g.kappa,
                              g.lam, ctypes.byref(opts), ctypes.byref(soa))
    assert rc == _lib.SBR_EARG and b"xi_guess" in L.sbr_last_error(engine._ctx)
    assert np.isnan(_lib.default_opts().xi_guess)
    # xi_guess is read only with SBR_FLAG_XI_GUESS: a zero-filled sbr_opts — what a
    # caller built against the round-4 header, or a memset, passes — sweeps with the defaults
    zero = _lib.Opts()
    rc = L.sbr_sweep_baseline(engine._ctx, P_(g.beta), P_(g.eta), P_(g.t_end), g.x0, P_(g.u), nb, nu, g.p, g.kappa,
                              g.lam, ctypes.byref(zero), ctypes.byref(soa))
    assert rc == _lib.SBR_OK
    ref = engine.sweep_baseline(g)
    for k in FIELDS:
        a, b = out[k].reshape(nb, nu), ref[k]
        assert np.array_equal(a.view(np.int64), b.view(np.int64)), k
