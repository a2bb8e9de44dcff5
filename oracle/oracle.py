"""ctypes binding to the CPU oracle (oracle/sbr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py — never by the product package.  See the header
of sbr_oracle.c for what is restated and how parity is pinned.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

_HERE = Path(__file__).resolve().parent
LIB_PATH = _HERE / "_build" / "libsbr_oracle.so"

_D = ctypes.c_double
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_P = ctypes.c_void_p


def build(force: bool = False) -> Path:
    if force or not LIB_PATH.exists():
        subprocess.run(["make", "-C", str(_HERE)], check=True, stdout=subprocess.DEVNULL)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.sbro_learn_logistic.restype = _I64
        L.sbro_learn_logistic.argtypes = [_D, _D, _D, _D, _D, _D, _I64, _P, _P, _I64, _P]
        L.sbro_equilibrium.restype = None
        L.sbro_equilibrium.argtypes = [_P, _P, _I64, _D, _D, _D, _D, _D, _D, _D, _I32, _P, _P, _P, _P, _P, _P, _P]
        L.sbro_equilibrium_paths.restype = None
        L.sbro_equilibrium_paths.argtypes = [_P, _P, _I64, _D, _D, _D, _D, _D, _D, _D, _I32] + [_P] * 9
        L.sbro_equilibrium_paths_pdf.restype = None
        L.sbro_equilibrium_paths_pdf.argtypes = [_P, _P, _P, _I64, _D, _D, _D, _D, _D, _D, _I32] + [_P] * 9
        L.sbro_sweep_baseline.restype = ctypes.c_int
        L.sbro_sweep_baseline.argtypes = [_P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _I32, _I32] + [_P] * 8
        L.sbro_apply_early_exit.restype = None
        L.sbro_apply_early_exit.argtypes = [_I64, _I64, _I32, _P, _P, _P, _P]
        L.sbro_detmath.restype = None
        L.sbro_detmath.argtypes = [_P, _P, _I64, _P, _P, _P]
        for name in ("sbro_sweep_hetero", "sbro_solve_social"):
            if hasattr(L, name):
                getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(_P)


EPS = float(np.finfo(np.float64).eps)


def learn_logistic(beta, t_end, x0=1e-4, t0=0.0, rtol=EPS, atol=EPS, maxiters=1_000_000, cap=1 << 16):
    t = np.empty(cap)
    G = np.empty(cap)
    stats = np.zeros(8, np.int64)
    n = lib().sbro_learn_logistic(beta, t0, t_end, x0, rtol, atol, maxiters, _ptr(t), _ptr(G), cap, _ptr(stats))
    if n < 0:
        raise RuntimeError(f"oracle knot buffer too small ({-n} needed)")
    return t[:n].copy(), G[:n].copy(), dict(naccept=int(stats[0]), nreject=int(stats[1]), status=int(stats[2]),
                                            t_switch=float(stats[4:5].view(np.float64)[0]),
                                            nswitch=int(stats[5]), nstiff=int(stats[6]))


def set_xi_guess(g: float = float("nan")) -> None:
    """compute_ξ's first iterate ξ_guess for the following calls (NaN: the default midpoint)."""
    L = lib()
    L.sbro_set_xi_guess.restype = None
    L.sbro_set_xi_guess.argtypes = [ctypes.c_double]
    L.sbro_set_xi_guess(g)


def equilibrium(t, G, beta, eta, t_end, u, p, kappa, lam, max_iters=100, paths=False):
    t = np.ascontiguousarray(t, np.float64)
    G = np.ascontiguousarray(G, np.float64)
    n = len(t)
    res = np.zeros(5)
    st = np.zeros(1, np.uint32)
    it = np.zeros(1, np.int32)
    hr_tau = np.zeros(n + 1) if paths else None
    hr_v = np.zeros(n + 1) if paths else None
    aw = np.zeros(n + 1) if paths else None
    nhr = np.zeros(1, np.int64)
    lib().sbro_equilibrium(_ptr(t), _ptr(G), n, beta, eta, t_end, u, p, kappa, lam, max_iters, _ptr(res),
                           _ptr(st), _ptr(it), _ptr(hr_tau), _ptr(hr_v), _ptr(aw), _ptr(nhr))
    out = dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
               iters=int(it[0]), n_hr=int(nhr[0]))
    if paths:
        k = int(nhr[0])
        out.update(hr_tau=hr_tau[:k], hr=hr_v[:k], aw=aw[:k])
    return out


def equilibrium_paths(t, G, beta, eta, t_end, u, p, kappa, lam, max_iters=100):
    """solve_equilibrium_baseline on caller knots with get_AW's three paths (AW_cum, AW_OUT,
    AW_IN on the hazard grid; n_hr = 0 after the hazard's BoundsError)."""
    t = np.ascontiguousarray(t, np.float64)
    G = np.ascontiguousarray(G, np.float64)
    n = len(t)
    res = np.zeros(5)
    st = np.zeros(1, np.uint32)
    it = np.zeros(1, np.int32)
    bufs = [np.full(n + 1, np.nan) for _ in range(5)]
    nhr = np.zeros(1, np.int64)
    lib().sbro_equilibrium_paths(_ptr(t), _ptr(G), n, beta, eta, t_end, u, p, kappa, lam, max_iters, _ptr(res),
                                 _ptr(st), _ptr(it), *[_ptr(b) for b in bufs], _ptr(nhr))
    k = int(nhr[0])
    out = dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
               iters=int(it[0]), n_hr=k)
    for name, b in zip(("hr_tau", "hr", "aw_cum", "aw_out", "aw_in"), bufs):
        out[name] = b[:k]
    return out


def equilibrium_paths_pdf(t, G, pdf, eta, t_end, u, p, kappa, lam, max_iters=100):
    """equilibrium_paths on an explicit learning pdf given by its knot values (hazard_rate(p, λ,
    LinearInterpolation(t, pdf), η); the social extension's (1 − G)·β·AW_{n−1})."""
    t = np.ascontiguousarray(t, np.float64)
    G = np.ascontiguousarray(G, np.float64)
    pdf = np.ascontiguousarray(pdf, np.float64)
    n = len(t)
    res = np.zeros(5)
    st = np.zeros(1, np.uint32)
    it = np.zeros(1, np.int32)
    bufs = [np.full(n + 1, np.nan) for _ in range(5)]
    nhr = np.zeros(1, np.int64)
    lib().sbro_equilibrium_paths_pdf(_ptr(t), _ptr(G), _ptr(pdf), n, eta, t_end, u, p, kappa, lam, max_iters,
                                     _ptr(res), _ptr(st), _ptr(it), *[_ptr(b) for b in bufs], _ptr(nhr))
    k = int(nhr[0])
    out = dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
               iters=int(it[0]), n_hr=k)
    for name, b in zip(("hr_tau", "hr", "aw_cum", "aw_out", "aw_in"), bufs):
        out[name] = b[:k]
    return out


def sweep_baseline(beta, eta, t_end, u, p, kappa, lam, x0=1e-4, max_iters=100, nthreads=0):
    beta = np.ascontiguousarray(beta, np.float64)
    eta = np.ascontiguousarray(np.broadcast_to(eta, beta.shape), np.float64)
    t_end = np.ascontiguousarray(np.broadcast_to(t_end, beta.shape), np.float64)
    u = np.ascontiguousarray(u, np.float64)
    nb, nu = len(beta), len(u)
    o = {k: np.empty(nb * nu) for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")}
    o["status"] = np.empty(nb * nu, np.uint32)
    o["iters"] = np.empty(nb * nu, np.int32)
    nk = np.empty(nb, np.int64)
    rc = lib().sbro_sweep_baseline(_ptr(beta), _ptr(eta), _ptr(t_end), x0, _ptr(u), nb, nu, p, kappa, lam,
                                   max_iters, nthreads, _ptr(o["xi"]), _ptr(o["tau_in_unc"]),
                                   _ptr(o["tau_out_unc"]), _ptr(o["aw_max"]), _ptr(o["tol"]), _ptr(o["status"]),
                                   _ptr(o["iters"]), _ptr(nk))
    if rc != 0:
        raise RuntimeError("oracle sweep failed")
    out = {k: v.reshape(nb, nu) for k, v in o.items()}
    out["n_knots"] = nk
    return out


def apply_early_exit(res: dict, threshold: int = 5) -> dict:
    r = {k: (v.copy() if isinstance(v, np.ndarray) else v) for k, v in res.items()}
    nb, nu = r["xi"].shape
    lib().sbro_apply_early_exit(nb, nu, threshold, _ptr(r["xi"]), _ptr(r["aw_max"]), _ptr(r["tol"]),
                                _ptr(r["status"]))
    return r


def fastpow(x, y):
    """FastPower.fastpower restated (include/sbr_detmath.h sbr_fastpow)."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(np.broadcast_to(y, x.shape), np.float64)
    out = np.empty(len(x))
    L = lib()
    L.sbro_fastpow.restype = None
    L.sbro_fastpow.argtypes = [_P, _P, _I64, _P]
    L.sbro_fastpow(_ptr(x), _ptr(y), len(x), _ptr(out))
    return out


def detmath(x, y):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    n = len(x)
    e, l, pw = np.empty(n), np.empty(n), np.empty(n)
    lib().sbro_detmath(_ptr(x), _ptr(y), n, _ptr(e), _ptr(l), _ptr(pw))
    return e, l, pw


def _hetero_sigs(L):
    L.sbro_sweep_hetero.restype = ctypes.c_int
    L.sbro_sweep_hetero.argtypes = [_I32, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _I32, _D, _I32] + [_P] * 8
    L.sbro_learn_hetero.restype = _I64
    L.sbro_learn_hetero.argtypes = [_P, _P, _I32, _D, _D, _P, _P, _I64, _P]


def learn_hetero(betas, dist, t_end, x0=1e-4, cap=1 << 16):
    L = lib()
    _hetero_sigs(L)
    betas = np.ascontiguousarray(betas, np.float64)
    dist = np.ascontiguousarray(dist, np.float64)
    K = len(betas)
    t = np.empty(cap)
    G = np.empty(cap * K)
    stats = np.zeros(8, np.int64)
    n = L.sbro_learn_hetero(_ptr(betas), _ptr(dist), K, t_end, x0, _ptr(t), _ptr(G), cap, _ptr(stats))
    if n < 0:
        raise RuntimeError("oracle hetero learning failed")
    return t[:n].copy(), G[: n * K].reshape(n, K).copy(), dict(naccept=int(stats[0]), nreject=int(stats[1]),
                                                                status=int(stats[2]),
                                                                t_switch=float(stats[4:5].view(np.float64)[0]),
                                                                nswitch=int(stats[5]), nstiff=int(stats[6]))


def sweep_hetero(betas, dist, eta, t_end, u, p, kappa, lam, x0=1e-4, max_iters=500, tolerance=1e-12, nthreads=0):
    """betas: [n_col, K] group rates per column; eta/t_end per column."""
    L = lib()
    _hetero_sigs(L)
    betas = np.ascontiguousarray(np.atleast_2d(betas), np.float64)
    n_col, K = betas.shape
    dist = np.ascontiguousarray(dist, np.float64)
    eta = np.ascontiguousarray(np.broadcast_to(eta, (n_col,)), np.float64)
    t_end = np.ascontiguousarray(np.broadcast_to(t_end, (n_col,)), np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    nu = len(u)
    o = {k: np.empty(n_col * nu) for k in ("xi", "aw_max", "tol")}
    o["status"] = np.empty(n_col * nu, np.uint32)
    o["iters"] = np.empty(n_col * nu, np.int32)
    o["tau_in_unc"] = np.empty(n_col * nu * K)
    o["tau_out_unc"] = np.empty(n_col * nu * K)
    nk = np.empty(n_col, np.int64)
    rc = L.sbro_sweep_hetero(K, _ptr(betas), _ptr(dist), _ptr(eta), _ptr(t_end), x0, _ptr(u), n_col, nu, p, kappa, lam,
                             max_iters, tolerance, nthreads, _ptr(o["xi"]), _ptr(o["aw_max"]), _ptr(o["tol"]),
                             _ptr(o["status"]), _ptr(o["iters"]), _ptr(o["tau_in_unc"]), _ptr(o["tau_out_unc"]),
                             _ptr(nk))
    if rc != 0:
        raise RuntimeError("oracle hetero sweep failed")
    out = {k: v.reshape(n_col, nu) for k, v in o.items() if k not in ("tau_in_unc", "tau_out_unc")}
    out["tau_in_unc"] = o["tau_in_unc"].reshape(n_col, nu, K)
    out["tau_out_unc"] = o["tau_out_unc"].reshape(n_col, nu, K)
    out["n_knots"] = nk
    return out


def _social_sigs(L):
    L.sbro_sweep_social.restype = ctypes.c_int
    L.sbro_sweep_social.argtypes = ([_P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _I32, _D, _I32, _I32, _I32]
                                    + [_P] * 9)


def sweep_social(beta, eta, u, p, kappa, lam, cmp, x0=1e-4, tol=1e-4, max_iter=500, bisect_max_iters=100,
                 nthreads=0, stats=False):
    """solve_equilibrium_social_learning (social_learning_solver.jl:63-263) over β columns × u.
    cmp: [n_beta, n_cmp] comparison grids (range(0, η_b, length=1000), :103)."""
    L = lib()
    _social_sigs(L)
    beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
    nb = len(beta)
    eta = np.ascontiguousarray(np.broadcast_to(eta, (nb,)), np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    nu = len(u)
    cmp = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(cmp), (nb, np.atleast_2d(cmp).shape[1])), np.float64)
    o = {k: np.empty(nb * nu) for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")}
    o["status"] = np.empty(nb * nu, np.uint32)
    o["iters"] = np.empty(nb * nu, np.int32)
    o["fp_iters"] = np.empty(nb * nu, np.int32)
    st = np.zeros(nb * nu * 4, np.int64) if stats else None
    rc = L.sbro_sweep_social(_ptr(beta), _ptr(eta), x0, _ptr(u), nb, nu, p, kappa, lam, _ptr(cmp), cmp.shape[1], tol,
                             max_iter, bisect_max_iters, nthreads, _ptr(o["xi"]), _ptr(o["tau_in_unc"]),
                             _ptr(o["tau_out_unc"]), _ptr(o["aw_max"]), _ptr(o["tol"]), _ptr(o["status"]),
                             _ptr(o["iters"]), _ptr(o["fp_iters"]), _ptr(st))
    if rc != 0:
        raise RuntimeError("oracle social sweep failed")
    out = {k: v.reshape(nb, nu) for k, v in o.items()}
    if stats:
        s = st.reshape(nb, nu, 4)
        out.update(n_knots=s[..., 0], n_accept=s[..., 1], n_reject=s[..., 2])
    return out


def social_point(beta, eta, u, p, kappa, lam, cmp, x0=1e-4, tol=1e-4, max_iter=500, cap=1 << 18):
    """One solve_equilibrium_social_learning point with the last iterate's
    learning knots (t, G), AW_{n-1} at those knots and HR grid τ̄ (to rebuild the plotted
    AW paths and the SolvedModel's learning_pdf / HR)."""
    L = lib()
    L.sbro_social_point.restype = _I64
    L.sbro_social_point.argtypes = [_D, _D, _D, _D, _D, _D, _D, _P, _I32, _D, _I32, _P, _P, _P, _P, _P, _P, _P, _I64,
                                    _P]
    cmp = np.ascontiguousarray(cmp, np.float64)
    res = np.zeros(5)
    st = np.zeros(1, np.uint32)
    fi = np.zeros(1, np.int32)
    t, G, tau, awo = np.empty(cap), np.empty(cap), np.empty(cap), np.empty(cap)
    ntau = np.zeros(1, np.int64)
    n = L.sbro_social_point(beta, eta, x0, u, p, kappa, lam, _ptr(cmp), len(cmp), tol, max_iter, _ptr(res), _ptr(st),
                            _ptr(fi), _ptr(t), _ptr(G), _ptr(tau), _ptr(awo), cap, _ptr(ntau))
    if n < 0:
        raise RuntimeError(f"oracle social path buffer too small ({-n} needed)")
    k = int(ntau[0])
    return dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
                fp_iters=int(fi[0]), t=t[:n].copy(), G=G[:n].copy(), hr_tau=tau[:k].copy(), aw_old=awo[:n].copy())


def sweep_interest(beta, eta, t_end, u, p, kappa, lam, r, delta, x0=1e-4, max_iters=100, nthreads=0):
    """solve_learning + solve_equilibrium_interest (interest_rate_solver.jl:51-150) +
    get_AW_functions_interest!(…).AW_max over β columns × u; rk_steps = value-function
    Tsit5 steps per point (0 when r = 0)."""
    L = lib()
    L.sbro_sweep_interest.restype = ctypes.c_int
    L.sbro_sweep_interest.argtypes = [_P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _D, _D, _I32, _I32] + [_P] * 8
    beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
    nb = len(beta)
    eta = np.ascontiguousarray(np.broadcast_to(eta, (nb,)), np.float64)
    t_end = np.ascontiguousarray(np.broadcast_to(t_end, (nb,)), np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    nu = len(u)
    o = {k: np.empty(nb * nu) for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")}
    o["status"] = np.empty(nb * nu, np.uint32)
    o["iters"] = np.empty(nb * nu, np.int32)
    o["rk_steps"] = np.empty(nb * nu, np.int64)
    rc = L.sbro_sweep_interest(_ptr(beta), _ptr(eta), _ptr(t_end), x0, _ptr(u), nb, nu, p, kappa, lam, r, delta,
                               max_iters, nthreads, _ptr(o["xi"]), _ptr(o["tau_in_unc"]), _ptr(o["tau_out_unc"]),
                               _ptr(o["aw_max"]), _ptr(o["tol"]), _ptr(o["status"]), _ptr(o["iters"]),
                               _ptr(o["rk_steps"]))
    if rc != 0:
        raise RuntimeError("oracle interest sweep failed")
    return {k: v.reshape(nb, nu) for k, v in o.items()}


def interest_point(beta, eta, t_end, u, p, kappa, lam, r, delta, x0=1e-4, cap=1 << 16):
    """One interest-rate equilibrium with its HR grid τ̄, HR(τ̄) and the value function
    V(τ̄) saved on that grid (value_function_solver.jl:66-112, saveat = HR knots)."""
    L = lib()
    L.sbro_interest_point.restype = _I64
    L.sbro_interest_point.argtypes = [_D, _D, _D, _D, _D, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P, _P, _I64, _P]
    res = np.zeros(5)
    st = np.zeros(1, np.uint32)
    tau, hr, V, aw = np.empty(cap), np.empty(cap), np.empty(cap), np.empty(cap)
    nv = np.zeros(1, np.int64)
    n = L.sbro_interest_point(beta, eta, t_end, x0, u, p, kappa, lam, r, delta, _ptr(res), _ptr(st), _ptr(tau),
                              _ptr(hr), _ptr(V), _ptr(aw), cap, _ptr(nv))
    if n < 0:
        raise RuntimeError(f"oracle interest path buffer too small ({-n} needed)")
    k = int(nv[0])
    return dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
                hr_tau=tau[:n].copy(), hr=hr[:n].copy(), V=V[:k].copy(), aw_cum=aw[:n].copy())


def hetero_point_paths(betas, dist, eta, t_end, u, p, kappa, lam, x0=1e-4, cap=1 << 16):
    """One heterogeneity equilibrium with the learning knots t, G [n, K], the per-group
    buffers, AW_total on the knots (get_AW_functions_hetero!, heterogeneity_solver.jl:386) and
    get_AW_hetero's per-group curves aw_out / aw_in [K, n] (:335-362)."""
    L = lib()
    L.sbro_hetero_point_paths.restype = _I64
    L.sbro_hetero_point_paths.argtypes = [_I32, _P, _P, _D, _D, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P, _P, _P, _P, _I64]
    betas = np.ascontiguousarray(betas, np.float64)
    dist = np.ascontiguousarray(dist, np.float64)
    K = len(dist)
    res = np.zeros(3)
    st = np.zeros(1, np.uint32)
    tin, tout = np.empty(K), np.empty(K)
    t, G, aw = np.empty(cap), np.empty(cap * K), np.empty(cap)
    awg = np.empty((2 * K, cap))
    n = L.sbro_hetero_point_paths(K, _ptr(betas), _ptr(dist), eta, t_end, x0, u, p, kappa, lam, _ptr(res), _ptr(st),
                                  _ptr(tin), _ptr(tout), _ptr(t), _ptr(G), _ptr(aw), _ptr(awg), cap)
    if n < 0:
        raise RuntimeError("oracle hetero point failed")
    return dict(xi=res[0], aw_max=res[1], tol=res[2], status=int(st[0]), tau_in_unc=tin, tau_out_unc=tout,
                t=t[:n].copy(), G=G[:n * K].reshape(n, K).copy(), aw_total=aw[:n].copy(),
                aw_out=awg[:K, :n].copy(), aw_in=awg[K:, :n].copy())


def hetero_equilibrium_knots(t, G, betas, dist, eta, t_end, u, p, kappa, lam):
    """solve_equilibrium_hetero(lr_hetero, econ) on caller knots t [n], G [n, K] for each u
    (sbro_hetero_equilibrium_knots): per-u arrays, per-group buffers [n_u, K], HR_k on the τ̄
    grid [K, n_hr] and, for one u, AW_total on the knots."""
    L = lib()
    L.sbro_hetero_equilibrium_knots.restype = None
    L.sbro_hetero_equilibrium_knots.argtypes = [_I32, _P, _P, _I64, _P, _P, _D, _D, _P, _I64, _D, _D, _D] + [_P] * 10
    t = np.ascontiguousarray(t, np.float64)
    G = np.ascontiguousarray(G, np.float64)
    betas = np.ascontiguousarray(betas, np.float64)
    dist = np.ascontiguousarray(dist, np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    n, K, nu = len(t), len(dist), len(u)
    o = {k: np.empty(nu) for k in ("xi", "aw_max", "tol")}
    o["status"] = np.empty(nu, np.uint32)
    o["iters"] = np.empty(nu, np.int32)
    tin, tout = np.empty((nu, K)), np.empty((nu, K))
    hr = np.full((K, n + 1), np.nan)
    nhr = np.zeros(1, np.int64)
    aw = np.full(n, np.nan) if nu == 1 else None
    L.sbro_hetero_equilibrium_knots(K, _ptr(t), _ptr(G), n, _ptr(betas), _ptr(dist), eta, t_end, _ptr(u), nu, p,
                                    kappa, lam, _ptr(o["xi"]), _ptr(o["aw_max"]), _ptr(o["tol"]), _ptr(o["status"]),
                                    _ptr(o["iters"]), _ptr(tin), _ptr(tout), _ptr(hr), _ptr(nhr), _ptr(aw))
    k = int(nhr[0])
    o.update(tau_in_unc=tin, tau_out_unc=tout, hr=hr[:, :k].copy(), n_hr=k, aw_total=aw)
    return o


def set_initdt_den(d: int = 6) -> None:
    """ode_determine_initdt's exponent 1/d (6: Tsit5's order + 1, the restatement's choice);
    other values only for tools/initdt_evidence.py."""
    L = lib()
    L.sbro_set_initdt_den.restype = None
    L.sbro_set_initdt_den.argtypes = [_I32]
    L.sbro_set_initdt_den(int(d))


def set_initdt(form: int = 0, den: int = 6) -> None:
    """form 0: (0.01/max(d₁,d₂))^(1/den); form 1: 10^(-(2 + log10(max(d₁,d₂)))/den), the
    published initdt.jl expression (tools/initdt_evidence.py)."""
    L = lib()
    L.sbro_set_initdt.restype = None
    L.sbro_set_initdt.argtypes = [_I32, _I32]
    L.sbro_set_initdt(int(form), int(den))


def set_initdt_ulps(k: int = 0) -> None:
    """Sensitivity probe: move the initial dt₁ by k ulps (tools/initdt_evidence.py)."""
    L = lib()
    L.sbro_set_initdt_ulps.restype = None
    L.sbro_set_initdt_ulps.argtypes = [_I32]
    L.sbro_set_initdt_ulps(int(k))
