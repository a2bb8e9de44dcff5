"""Host-side mirror of the reference's learning/solver call surface, backed by
libsbr's gfx950 kernels.

Reference call surface → here:
  solve_learning(::LearningParameters)              learning.jl:109   → solve_learning(lp)
  solve_equilibrium_baseline(lr, econ)              solver.jl:413     → solve_equilibrium_baseline(lr, econ)
  get_AW_functions!(result)                         solver.jl:553     → get_AW_functions(result)
  the Fig 4 / Fig 5 double loops                    1_baseline.jl:151-192, 224-267
                                                                      → Engine.sweep_baseline(grid)
  solve_equilibrium_social_learning(model; tol, max_iter)
                                                    social_learning_solver.jl:63
                                                                      → solve_equilibrium_social_learning(model)
                                                                        / Engine.sweep_social(...)
  solve_SInetwork_hetero + solve_equilibrium_hetero heterogeneity_*.jl → Engine.sweep_hetero / hetero_point_paths
  solve_equilibrium_interest(lr, econ, model)       interest_rate_solver.jl:51
                                                                      → Engine.sweep_interest / interest_point_paths
There is no CPU fallback: without libsbr.so or a GPU every call raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import ArgumentError, SBRNativeError, check
from .grids import BaselineGrid, julia_range
from .model import (EconomicParameters, EconomicParametersInterest, LearningParameters, ModelParameters,
                    ModelParametersHetero, ModelParametersInterest)

_P = ctypes.c_void_p

RESULT_FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")
# learning-level status bits a sweep point carries from its column's ODE solve
_LEARN_BITS = (_lib.STATUS["SBR_ODE_MAXITERS"] | _lib.STATUS["SBR_STIFF_SWITCH"] | _lib.STATUS["SBR_ODE_FAILED"]
               | _lib.STATUS["SBR_KNOT_OVERFLOW"])


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(_P)


_F64, _I32, _I64 = "float64", "int32", "int64"


def _dptr(t, name: str, kind: str, numel: int | None = None, optional: bool = False):
    """data_ptr() of a device tensor handed to a *_dev entry point, after the checks the
    kernels cannot make: a contiguous CUDA tensor of the right dtype holding at least
    ``numel`` elements.  Anything else raises ArgumentError (never a silent OOB access)."""
    if t is None:
        if optional:
            return None
        raise ArgumentError(f"{name}: a device tensor is required")
    import torch
    want = {_F64: (torch.float64,), _I32: (torch.int32, getattr(torch, "uint32", torch.int32)),
            _I64: (torch.int64,)}[kind]
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise ArgumentError(f"{name}: expected a CUDA tensor")
    if t.dtype not in want:
        raise ArgumentError(f"{name}: expected dtype {kind}, got {t.dtype}")
    if not t.is_contiguous():
        raise ArgumentError(f"{name}: tensor must be contiguous")
    if numel is not None and t.numel() < numel:
        raise ArgumentError(f"{name}: needs at least {numel} elements, has {t.numel()}")
    return t.data_ptr()


def _out_ptrs(out: dict, fields, n: int, required=()):
    """SoA result pointers from ``out`` (missing / None entries are NULL unless required)."""
    ptrs = []
    for k in fields:
        kind = _I32 if k in ("status", "iters", "fp_iters") else (_I64 if k == "rk_steps" else _F64)
        ptrs.append(_dptr(out.get(k), f"out[{k!r}]", kind, n, optional=k not in required))
    return ptrs


def host_result_views(out: dict, n: int) -> dict:
    """Flat views of a caller's host result arrays for sbr_sweep_baseline: float64 RESULT_FIELDS,
    uint32 ``status`` and optional int32 ``iters``, each C-contiguous with ``n`` elements.
    Anything else raises ArgumentError before the C call (no write past a caller's array)."""
    want = {**{k: np.float64 for k in RESULT_FIELDS}, "status": np.uint32, "iters": np.int32}
    views = {}
    for k, dt in want.items():
        v = out.get(k)
        if v is None and k == "iters":
            views[k] = None
            continue
        if not isinstance(v, np.ndarray) or v.dtype != dt or v.size != n or not v.flags["C_CONTIGUOUS"]:
            raise ArgumentError(f"out[{k!r}] must be a C-contiguous {np.dtype(dt).name} array of {n}")
        views[k] = v.reshape(-1)
    return views


class Engine:
    """One libsbr context: one HIP device (``device``), or — with ``n_gpus`` /
    ``devices`` — an n-device context whose host-pointer sweeps fan out over the GPUs
    inside libsbr (one host thread per GPU, each GPU's results over its own PCIe link;
    sbr_init_multi)."""

    def __init__(self, device: int | None = None, n_gpus: int | None = None, devices=None):
        L = _lib.load()
        ctx = _P()
        self._multi = n_gpus is not None or devices is not None
        if self._multi:
            devs = None if devices is None else (ctypes.c_int * len(devices))(*devices)
            n = len(devices) if devices is not None else int(n_gpus)
            rc = L.sbr_init_multi(n, devs, ctypes.byref(ctx))
            if rc != 0:
                raise SBRNativeError(f"sbr_init_multi(n_gpus={n}) failed ({rc})")
            self.device = devices[0] if devices is not None else 0
        else:
            if device is None:
                device = int(os.environ.get("LOCAL_RANK", "0"))
            self.device = device
            rc = L.sbr_init(device, ctypes.byref(ctx))
            if rc != 0:
                raise SBRNativeError(f"sbr_init(device={device}) failed ({rc}): no usable HIP device")
        self._ctx = ctx
        self._L = L
        self._knot_opts = {}  # sbr_opts per bisect_max_iters of equilibrium_on_knots (per-call latency)

    @property
    def n_gpus(self) -> int:
        """Devices this context sweeps over (sbr_multi_size)."""
        return int(self._L.sbr_multi_size(self._ctx))

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.sbr_free(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ sweeps
    def sweep_baseline(self, grid: BaselineGrid, early_exit: int = 0, max_iters: int = 100,
                       knot_capacity: int = 65536, with_iters: bool = True, exhaustive: bool = False,
                       flags: int = 0, out: dict | None = None) -> dict:
        """Every (β, u) of ``grid`` through learning → HR → buffers → bisection
        → AW_max.  Returns [n_beta, n_u] arrays (row i = β_i).  ``early_exit=5``
        applies the reference's 5-consecutive-no-run rule as a post-pass.  ``out``: the
        caller's result arrays (as the reference's scripts fill matrices they allocated
        once), reused across calls; float64 RESULT_FIELDS, uint32 ``status``, optional int32
        ``iters``, each C-contiguous with n_beta·n_u elements."""
        nb, nu = grid.shape
        if out is None:
            out = {k: np.empty(nb * nu) for k in RESULT_FIELDS}
            out["status"] = np.empty(nb * nu, np.uint32)
            out["iters"] = np.empty(nb * nu, np.int32) if with_iters else None
        else:
            out = host_result_views(out, nb * nu)
        soa = _lib.ResultSoA(*[_ptr(out[k]) for k in (*RESULT_FIELDS, "status", "iters")])
        opts = _lib.default_opts(early_exit_nan_run=early_exit, bisect_max_iters=max_iters,
                                 knot_capacity=knot_capacity,
                                 flags=flags | (_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0))
        rc = self._L.sbr_sweep_baseline(self._ctx, _ptr(grid.beta), _ptr(grid.eta), _ptr(grid.t_end), grid.x0,
                                        _ptr(grid.u), nb, nu, grid.p, grid.kappa, grid.lam, ctypes.byref(opts),
                                        ctypes.byref(soa))
        check(rc, self._ctx, "sbr_sweep_baseline")
        return {k: (v.reshape(nb, nu) if v is not None else None) for k, v in out.items()}

    def sweep_baseline_dev(self, beta, eta, t_end, u, p, kappa, lam, x0, out: dict, stream: int | None = None,
                           max_iters: int = 100, knot_capacity: int = 65536, exhaustive: bool = False,
                           flags: int = 0):
        """Device-pointer variant on torch tensors (float64 cuda) — no host sync.
        ``out`` holds preallocated tensors xi/tau_in_unc/tau_out_unc/aw_max/tol
        (float64), status (int32 viewed as uint32) and optional iters (int32)."""
        nb, nu = beta.numel(), u.numel()
        soa = _lib.ResultSoA(*_out_ptrs(out, (*RESULT_FIELDS, "status", "iters"), nb * nu,
                                        required=(*RESULT_FIELDS, "status")))
        opts = _lib.default_opts(early_exit_nan_run=0, bisect_max_iters=max_iters, knot_capacity=knot_capacity,
                                 flags=(_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0) | flags)
        rc = self._L.sbr_sweep_baseline_dev(self._ctx, stream, _dptr(beta, "beta", _F64),
                                            _dptr(eta, "eta", _F64, nb), _dptr(t_end, "t_end", _F64, nb),
                                            x0, _dptr(u, "u", _F64), nb, nu, p, kappa, lam, ctypes.byref(opts),
                                            ctypes.byref(soa))
        check(rc, self._ctx, "sbr_sweep_baseline_dev")

    def sweep_baseline_batch_dev(self, beta, eta, t_end, u, p, kappa, lam, x0, out: dict, stream: int | None = None,
                                 max_iters: int = 100, knot_capacity: int = 65536, flags: int = 0):
        """Pipelined sweep of several grids on torch tensors (float64 cuda):
        ``beta``/``eta``/``t_end`` are [n_batch, n_beta]; every ``out`` tensor
        is [n_batch, n_beta * n_u] (see sbr_sweep_baseline_batch_dev)."""
        nbat, nb = beta.shape
        nu = u.numel()
        if tuple(eta.shape) != (nbat, nb) or tuple(t_end.shape) != (nbat, nb):
            raise ArgumentError("eta and t_end must be [n_batch, n_beta] like beta")
        soa = _lib.ResultSoA(*_out_ptrs(out, (*RESULT_FIELDS, "status", "iters"), nbat * nb * nu,
                                        required=(*RESULT_FIELDS, "status")))
        opts = _lib.default_opts(early_exit_nan_run=0, bisect_max_iters=max_iters, knot_capacity=knot_capacity,
                                 flags=flags)
        rc = self._L.sbr_sweep_baseline_batch_dev(self._ctx, stream, nbat, _dptr(beta, "beta", _F64),
                                                  _dptr(eta, "eta", _F64), _dptr(t_end, "t_end", _F64), x0,
                                                  _dptr(u, "u", _F64), nb, nu, p, kappa, lam,
                                                  ctypes.byref(opts), ctypes.byref(soa))
        check(rc, self._ctx, "sbr_sweep_baseline_batch_dev")

    def batch_reserve(self, n_batch: int, n_beta: int, knot_capacity: int = 65536):
        """Allocate now the workspaces a later ``sweep_baseline_batch_dev`` of ``n_batch`` grids of
        ``n_beta`` columns uses (sbr_batch_reserve): the batch call then allocates nothing."""
        opts = _lib.default_opts(knot_capacity=knot_capacity)
        check(self._L.sbr_batch_reserve(self._ctx, int(n_batch), int(n_beta), ctypes.byref(opts)), self._ctx,
              "sbr_batch_reserve")

    def set_batch_workspace(self, nbytes: int):
        """Budget in bytes for the baseline batch's learning workspaces (0 = the default, 40 % of
        free HBM); it caps the grids learned per launch (sbr_set_batch_workspace)."""
        check(self._L.sbr_set_batch_workspace(self._ctx, int(nbytes)), self._ctx, "sbr_set_batch_workspace")

    def batch_wait(self, stream: int | None, k: int):
        """Make ``stream`` wait until grid ``k`` of the last batch call has its results
        (sbr_batch_wait): ship grid k while the rest of the batch is still being swept."""
        check(self._L.sbr_batch_wait(self._ctx, stream, int(k)), self._ctx, "sbr_batch_wait")

    def learn_baseline(self, beta, eta, t_end, x0=1e-4, stop_after_eta=False, cap=65536, tol=None):
        beta = np.ascontiguousarray(beta, np.float64)
        nb = len(beta)
        eta = np.ascontiguousarray(np.broadcast_to(eta, beta.shape), np.float64)
        t_end = np.ascontiguousarray(np.broadcast_to(t_end, beta.shape), np.float64)
        T = np.zeros((nb, cap))
        G = np.zeros((nb, cap))
        nk = np.zeros(nb, np.int32)
        st = np.zeros(nb, np.uint32)
        opts = _lib.default_opts(knot_capacity=cap)
        if tol is not None:  # solve_SIhomogeneous(…; tol): reltol = abstol = tol (learning.jl:41-51)
            opts.ode_reltol = opts.ode_abstol = float(tol)
        rc = self._L.sbr_learn_baseline(self._ctx, _ptr(beta), _ptr(eta), _ptr(t_end), x0, nb, int(stop_after_eta),
                                        ctypes.byref(opts), _ptr(T), _ptr(G), cap, _ptr(nk), _ptr(st))
        check(rc, self._ctx, "sbr_learn_baseline")
        return [(T[i, : nk[i]].copy(), G[i, : nk[i]].copy(), int(st[i])) for i in range(nb)]

    def solve_point_paths(self, beta, eta, t_end, u, p, kappa, lam, x0=1e-4, cap=65536):
        res = np.zeros(5)
        st = np.zeros(1, np.uint32)
        tau = np.zeros(cap)
        hr = np.zeros(cap)
        aw = np.zeros(cap)
        nt = np.zeros(1, np.int64)
        opts = _lib.default_opts(knot_capacity=cap)
        rc = self._L.sbr_solve_point_paths(self._ctx, beta, eta, t_end, x0, u, p, kappa, lam, ctypes.byref(opts),
                                           _ptr(res), _ptr(st), _ptr(tau), _ptr(hr), _ptr(aw), cap, _ptr(nt))
        check(rc, self._ctx, "sbr_solve_point_paths")
        k = int(nt[0])
        return dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4],
                    status=int(st[0]), tau=tau[:k].copy(), hr=hr[:k].copy(), aw_cum=aw[:k].copy())

    def equilibrium_on_knots(self, t, G, beta, eta, t_end, u, p, kappa, lam, max_iters: int = 100,
                             paths: bool = True, exhaustive: bool = False, xi_guess: float | None = None,
                             pdf=None) -> dict:
        """solve_equilibrium_baseline(lr, econ) + get_AW_functions!(r) (solver.jl:413-462, 553-576)
        on the learning knots the caller holds (t, G = lr.learning_cdf's knots and values) for each
        u — no learning ODE (sbr_equilibrium_on_knots).  The knots and the hazard path stay on the
        GPU while (t, G, β, η, p, λ) repeat, so a per-u loop over one LearningResults uploads only
        u.  Returns the SoA fields ([n_u] arrays); with ``paths`` (one u) also the hazard grid
        ``tau``, ``hr`` and ``aw_cum`` / ``aw_out`` / ``aw_in`` on it (NaN without a run).
        ``xi_guess``: compute_ξ's first iterate (solver.jl:413,441; None = the midpoint).
        ``pdf``: the learning pdf's values on the knots (sbr_equilibrium_on_knots_pdf; ``beta`` is
        then unused) — the social extension's (1 − G)·β·AW_{n−1}; None = βG(1 − G)."""
        t = t if (isinstance(t, np.ndarray) and t.dtype == np.float64 and t.flags.c_contiguous) else \
            np.ascontiguousarray(t, np.float64)
        G = G if (isinstance(G, np.ndarray) and G.dtype == np.float64 and G.flags.c_contiguous) else \
            np.ascontiguousarray(G, np.float64)
        if len(G) != len(t):
            raise ArgumentError("t and G must have the same length")
        u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        n, nu = len(t), len(u)
        if paths and nu != 1:
            raise ArgumentError("paths need a single u")
        res = np.empty(6 * nu)  # xi, tau_in_unc, tau_out_unc, aw_max, tol, then status / iters (int32)
        st_it = res[5 * nu:].view(np.int32)
        base = res.ctypes.data
        soa = _lib.ResultSoA(base, base + 8 * nu, base + 16 * nu, base + 24 * nu, base + 32 * nu, base + 40 * nu,
                             base + 44 * nu)
        key = (max_iters, exhaustive, xi_guess)
        opts = self._knot_opts.get(key)
        if opts is None:
            if len(self._knot_opts) > 64:  # per-call guesses: keep the cache bounded
                self._knot_opts = {}
            opts = self._knot_opts[key] = _lib.default_opts(
                bisect_max_iters=max_iters,
                flags=(_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0)
                | (_lib.SBR_FLAG_XI_GUESS if xi_guess is not None else 0),
                xi_guess=float("nan") if xi_guess is None else float(xi_guess))
        cap = n + 1
        nt = ctypes.c_int64()
        if paths:
            pbuf = np.empty(5 * cap)
            pb = pbuf.ctypes.data
            pp = (pb, pb + 8 * cap, pb + 16 * cap, pb + 24 * cap, pb + 32 * cap)
        else:
            pp = (None,) * 5
        if pdf is None:
            rc = self._L.sbr_equilibrium_on_knots(self._ctx, t.ctypes.data, G.ctypes.data, n, beta, eta, t_end,
                                                  u.ctypes.data, nu, p, kappa, lam, ctypes.byref(opts),
                                                  ctypes.byref(soa), *pp, cap, ctypes.byref(nt))
            check(rc, self._ctx, "sbr_equilibrium_on_knots")
        else:
            pdf = np.ascontiguousarray(pdf, np.float64)
            if len(pdf) != n:
                raise ArgumentError("t and pdf must have the same length")
            rc = self._L.sbr_equilibrium_on_knots_pdf(self._ctx, t.ctypes.data, G.ctypes.data, pdf.ctypes.data, n,
                                                      eta, t_end, u.ctypes.data, nu, p, kappa, lam,
                                                      ctypes.byref(opts), ctypes.byref(soa), *pp, cap,
                                                      ctypes.byref(nt))
            check(rc, self._ctx, "sbr_equilibrium_on_knots_pdf")
        out = dict(xi=res[:nu], tau_in_unc=res[nu:2 * nu], tau_out_unc=res[2 * nu:3 * nu],
                   aw_max=res[3 * nu:4 * nu], tol=res[4 * nu:5 * nu], status=st_it[:nu].view(np.uint32),
                   iters=st_it[nu:2 * nu])
        if paths:
            k = nt.value
            pv = pbuf.reshape(5, cap)
            out.update(tau=pv[0, :k], hr=pv[1, :k], aw_cum=pv[2, :k], aw_out=pv[3, :k], aw_in=pv[4, :k])
        return out

    def hetero_equilibrium_on_knots(self, t, G, betas, dist, eta, t_end, u, p, kappa, lam,
                                    paths: bool = True, exhaustive: bool = False) -> dict:
        """solve_equilibrium_hetero(lr_hetero, econ) + get_AW_functions_hetero! on the knots a
        LearningResultsHetero holds (t [n], G [n, K] = the learning_cdfs' values) for each u — no
        learning ODE (sbr_hetero_equilibrium_on_knots; knots, CDFs and the K hazards stay on the
        GPU while the inputs repeat).  Per-u arrays, buffers [n_u, K]; with ``paths`` (one u) HR_k
        on the τ̄ grid [K, n_tau], AW_total on the knots and get_AW_hetero's per-group curves
        aw_out / aw_in [K, n] (heterogeneity_solver.jl:335-362; NaN without a run)."""
        t = np.ascontiguousarray(t, np.float64)
        G = np.ascontiguousarray(G, np.float64)
        betas = np.ascontiguousarray(betas, np.float64)
        dist = np.ascontiguousarray(dist, np.float64)
        u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        n, K, nu = len(t), len(dist), len(u)
        if G.shape != (n, K) or betas.shape != (K,):
            raise ArgumentError("G must be [n_knots, K] and betas [K]")
        if paths and nu != 1:
            raise ArgumentError("paths need a single u")
        out = {k: np.empty(nu) for k in ("xi", "aw_max", "tol")}
        out["status"] = np.empty(nu, np.uint32)
        out["iters"] = np.empty(nu, np.int32)
        tin, tout = np.empty((nu, K)), np.empty((nu, K))
        soa = _lib.ResultSoA(_ptr(out["xi"]), None, None, _ptr(out["aw_max"]), _ptr(out["tol"]), _ptr(out["status"]),
                             _ptr(out["iters"]))
        cap = n + 1
        hr = np.empty((K, cap)) if paths else None
        aw = np.empty(cap) if paths else None
        awg = np.empty((2 * K, cap)) if paths else None
        nt = ctypes.c_int64()
        opts = _lib.default_opts(early_exit_nan_run=0, flags=_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0)
        rc = self._L.sbr_hetero_equilibrium_on_knots(self._ctx, K, _ptr(t), _ptr(G), n, _ptr(betas), _ptr(dist), eta,
                                                     t_end, _ptr(u), nu, p, kappa, lam, ctypes.byref(opts),
                                                     ctypes.byref(soa), _ptr(tin), _ptr(tout), _ptr(hr), _ptr(aw),
                                                     _ptr(awg), cap, ctypes.byref(nt))
        check(rc, self._ctx, "sbr_hetero_equilibrium_on_knots")
        out.update(tau_in_unc=tin, tau_out_unc=tout)
        if paths:
            k = nt.value
            out.update(hr=hr[:, :k], aw_total=aw[:n], aw_out=awg[:K, :n], aw_in=awg[K:, :n], n_tau=k)
        return out

    def sweep_hetero(self, betas, dist, eta, t_end, u, p, kappa, lam, x0=1e-4, knot_capacity: int = 16384,
                     with_groups: bool = True, exhaustive: bool = False) -> dict:
        """Heterogeneity sweep: ``betas`` [n_col, K] group rates per column,
        ``eta``/``t_end`` per column, every u.  Returns [n_col, n_u] arrays and,
        with ``with_groups``, per-group buffers [n_col, n_u, K]."""
        betas = np.ascontiguousarray(np.atleast_2d(betas), np.float64)
        n_col, K = betas.shape
        dist = np.ascontiguousarray(dist, np.float64)
        eta = np.ascontiguousarray(np.broadcast_to(eta, (n_col,)), np.float64)
        t_end = np.ascontiguousarray(np.broadcast_to(t_end, (n_col,)), np.float64)
        u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        nu = len(u)
        out = {k: np.empty(n_col * nu) for k in ("xi", "aw_max", "tol")}
        out["status"] = np.empty(n_col * nu, np.uint32)
        out["iters"] = np.empty(n_col * nu, np.int32)
        tin = np.empty(n_col * nu * K) if with_groups else None
        tout = np.empty(n_col * nu * K) if with_groups else None
        soa = _lib.ResultSoA(_ptr(out["xi"]), None, None, _ptr(out["aw_max"]), _ptr(out["tol"]),
                             _ptr(out["status"]), _ptr(out["iters"]))
        opts = _lib.default_opts(knot_capacity=knot_capacity, flags=_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0)
        rc = self._L.sbr_sweep_hetero(self._ctx, K, _ptr(betas), _ptr(dist), _ptr(eta), _ptr(t_end), x0, _ptr(u),
                                      n_col, nu, p, kappa, lam, ctypes.byref(opts), ctypes.byref(soa), _ptr(tin),
                                      _ptr(tout))
        check(rc, self._ctx, "sbr_sweep_hetero")
        res = {k: v.reshape(n_col, nu) for k, v in out.items()}
        if with_groups:
            res["tau_in_unc"] = tin.reshape(n_col, nu, K)
            res["tau_out_unc"] = tout.reshape(n_col, nu, K)
        return res

    def sweep_hetero_dev(self, K, betas, dist, eta, t_end, u, p, kappa, lam, x0, out: dict,
                         stream: int | None = None, knot_capacity: int = 16384, flags: int = 0):
        """Device-pointer hetero sweep on torch tensors (no host sync)."""
        n_col, nu = eta.numel(), u.numel()
        xi, aw, tl, st, it = _out_ptrs(out, ("xi", "aw_max", "tol", "status", "iters"), n_col * nu,
                                       required=("xi", "aw_max", "tol", "status"))
        soa = _lib.ResultSoA(xi, None, None, aw, tl, st, it)
        opts = _lib.default_opts(knot_capacity=knot_capacity, flags=flags)
        rc = self._L.sbr_sweep_hetero_dev(self._ctx, stream, K, _dptr(betas, "betas", _F64, n_col * K),
                                          _dptr(dist, "dist", _F64, K), _dptr(eta, "eta", _F64),
                                          _dptr(t_end, "t_end", _F64, n_col), x0, _dptr(u, "u", _F64), n_col, nu, p,
                                          kappa, lam, ctypes.byref(opts), ctypes.byref(soa), None, None)
        check(rc, self._ctx, "sbr_sweep_hetero_dev")

    def sweep_hetero_batch_dev(self, K, betas, dist, eta, t_end, u, p, kappa, lam, x0, out: dict,
                               stream: int | None = None, knot_capacity: int = 16384, flags: int = 0):
        """Pipelined hetero sweep of several grids on torch tensors (see
        sbr_sweep_hetero_batch_dev): ``betas`` [n_batch, n_col, K], ``eta``/``t_end``
        [n_batch, n_col], every ``out`` tensor [n_batch, n_col * n_u]."""
        nbat, n_col = eta.shape
        nu = u.numel()
        if tuple(betas.shape) != (nbat, n_col, K) or tuple(t_end.shape) != (nbat, n_col):
            raise ArgumentError("betas must be [n_batch, n_col, K] and t_end [n_batch, n_col]")
        xi, aw, tl, st, it = _out_ptrs(out, ("xi", "aw_max", "tol", "status", "iters"), nbat * n_col * nu,
                                       required=("xi", "aw_max", "tol", "status"))
        soa = _lib.ResultSoA(xi, None, None, aw, tl, st, it)
        opts = _lib.default_opts(knot_capacity=knot_capacity, flags=flags)
        rc = self._L.sbr_sweep_hetero_batch_dev(self._ctx, stream, nbat, K, _dptr(betas, "betas", _F64),
                                                _dptr(dist, "dist", _F64, K), _dptr(eta, "eta", _F64),
                                                _dptr(t_end, "t_end", _F64), x0, _dptr(u, "u", _F64), n_col, nu, p,
                                                kappa, lam, ctypes.byref(opts), ctypes.byref(soa), None, None)
        check(rc, self._ctx, "sbr_sweep_hetero_batch_dev")

    def sweep_social(self, beta, eta, u, p, kappa, lam, cmp=None, x0=1e-4, tol=1e-4, max_iter=500,
                     knot_capacity: int = 0, workspace_bytes: int | None = None) -> dict:
        """Social-learning sweep (social_learning_solver.jl:63-263) over β columns × u.
        ``cmp`` [n_beta, n_cmp]: the comparison grids range(0, η_b, length=1000) (built
        with Julia's range semantics when omitted).  Returns [n_beta, n_u] arrays."""
        beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
        nb = len(beta)
        eta = np.ascontiguousarray(np.broadcast_to(eta, (nb,)), np.float64)
        u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        nu = len(u)
        if cmp is None:
            cmp = np.stack([julia_range(0.0, float(e), 1000) for e in eta])
        cmp = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(cmp), (nb, np.atleast_2d(cmp).shape[1])),
                                   np.float64)
        out = {k: np.empty(nb * nu) for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")}
        out["status"] = np.empty(nb * nu, np.uint32)
        out["iters"] = np.empty(nb * nu, np.int32)
        out["fp_iters"] = np.empty(nb * nu, np.int32)
        out["rk_steps"] = np.empty(nb * nu, np.int64)
        soa = _lib.ResultSoA(*[_ptr(out[k]) for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status",
                                                      "iters")])
        opts = _lib.default_opts(pad=knot_capacity)
        if workspace_bytes is not None:
            check(self._L.sbr_set_social_workspace(self._ctx, int(workspace_bytes)), self._ctx,
                  "sbr_set_social_workspace")
        rc = self._L.sbr_sweep_social(self._ctx, _ptr(beta), _ptr(eta), x0, _ptr(u), nb, nu, p, kappa, lam, _ptr(cmp),
                                      cmp.shape[1], tol, max_iter, ctypes.byref(opts), ctypes.byref(soa),
                                      _ptr(out["fp_iters"]), _ptr(out["rk_steps"]))
        check(rc, self._ctx, "sbr_sweep_social")
        return {k: v.reshape(nb, nu) for k, v in out.items()}

    def sweep_social_dev(self, beta, eta, u, p, kappa, lam, cmp, x0, out: dict, tol=1e-4, max_iter=500,
                         stream: int | None = None, knot_capacity: int = 0, flags: int = 0):
        """Device-pointer social sweep on torch tensors (enqueue only)."""
        nb, nu = beta.numel(), u.numel()
        soa = _lib.ResultSoA(*_out_ptrs(out, (*RESULT_FIELDS, "status", "iters"), nb * nu,
                                        required=(*RESULT_FIELDS, "status")))
        opts = _lib.default_opts(pad=knot_capacity, flags=flags)
        fp, rk = _out_ptrs(out, ("fp_iters", "rk_steps"), nb * nu)
        n_cmp = cmp.shape[-1]
        rc = self._L.sbr_sweep_social_dev(self._ctx, stream, _dptr(beta, "beta", _F64), _dptr(eta, "eta", _F64, nb),
                                          x0, _dptr(u, "u", _F64), nb, nu, p, kappa, lam,
                                          _dptr(cmp, "cmp", _F64, nb * n_cmp), n_cmp, tol, max_iter,
                                          ctypes.byref(opts), ctypes.byref(soa), fp, rk)
        check(rc, self._ctx, "sbr_sweep_social_dev")

    def sweep_interest(self, beta, eta, t_end, u, p, kappa, lam, r, delta, x0=1e-4, max_iters: int = 100,
                       knot_capacity: int = 65536) -> dict:
        """Interest-rate extension over β columns × u (interest_rate_solver.jl:51-150 +
        get_AW_functions_interest!): the value function on the HR grid and buffers from
        h − rV (r > 0), the baseline for r = 0.  Returns [n_beta, n_u] arrays incl.
        rk_steps (value-function Tsit5 steps per point)."""
        beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
        nb = len(beta)
        eta = np.ascontiguousarray(np.broadcast_to(eta, (nb,)), np.float64)
        t_end = np.ascontiguousarray(np.broadcast_to(t_end, (nb,)), np.float64)
        u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        nu = len(u)
        out = {k: np.empty(nb * nu) for k in RESULT_FIELDS}
        out["status"] = np.empty(nb * nu, np.uint32)
        out["iters"] = np.empty(nb * nu, np.int32)
        out["rk_steps"] = np.empty(nb * nu, np.int64)
        soa = _lib.ResultSoA(*[_ptr(out[k]) for k in (*RESULT_FIELDS, "status", "iters")])
        opts = _lib.default_opts(early_exit_nan_run=0, bisect_max_iters=max_iters, knot_capacity=knot_capacity)
        rc = self._L.sbr_sweep_interest(self._ctx, _ptr(beta), _ptr(eta), _ptr(t_end), x0, _ptr(u), nb, nu, p, kappa,
                                        lam, r, delta, ctypes.byref(opts), ctypes.byref(soa), _ptr(out["rk_steps"]))
        check(rc, self._ctx, "sbr_sweep_interest")
        return {k: v.reshape(nb, nu) for k, v in out.items()}

    def social_point_paths(self, beta, eta, u, p, kappa, lam, cmp=None, x0=1e-4, tol=1e-4, max_iter=500,
                           cap=1 << 20) -> dict:
        """One social-learning fixed point with the learning knots (t, G) of the returned
        SolvedModel and AW_{n-1} at those knots (the forcing of its learning_pdf,
        social_learning_dynamics.jl:98-114) — what scripts/4_social_learning.jl plots."""
        if cmp is None:
            cmp = julia_range(0.0, float(eta), 1000)
        cmp = np.ascontiguousarray(cmp, np.float64)
        res = np.zeros(5)
        st = np.zeros(1, np.uint32)
        fp = np.zeros(1, np.int32)
        t, G, awo = np.empty(cap), np.empty(cap), np.empty(cap)
        nk = ctypes.c_int64()
        opts = _lib.default_opts()
        rc = self._L.sbr_social_point_paths(self._ctx, beta, eta, x0, u, p, kappa, lam, _ptr(cmp), len(cmp), tol,
                                            max_iter, ctypes.byref(opts), _ptr(res), _ptr(st), _ptr(fp), _ptr(t),
                                            _ptr(G), _ptr(awo), cap, ctypes.byref(nk))
        check(rc, self._ctx, "sbr_social_point_paths")
        n = nk.value
        return dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
                    fp_iters=int(fp[0]), t=t[:n].copy(), G=G[:n].copy(), aw_old=awo[:n].copy())

    def learn_hetero(self, betas, dist, t_end, x0=1e-4, cap=16384) -> dict:
        """solve_SInetwork_hetero (heterogeneity_learning.jl:49-94) for n_col columns: the shared
        knot grid t [n_col, cap] and group CDFs G [n_col, cap, K] (row c valid to n_knots[c])."""
        dist = np.ascontiguousarray(dist, np.float64)
        K = len(dist)
        betas = np.ascontiguousarray(np.atleast_2d(betas), np.float64)
        nc = betas.shape[0]
        assert betas.shape[1] == K
        t_end = np.ascontiguousarray(np.broadcast_to(t_end, (nc,)), np.float64)
        t, G = np.empty((nc, cap)), np.empty((nc, cap, K))
        nk, st = np.zeros(nc, np.int32), np.zeros(nc, np.uint32)
        opts = _lib.default_opts(early_exit_nan_run=0, knot_capacity=cap)
        rc = self._L.sbr_learn_hetero(self._ctx, K, _ptr(betas), _ptr(dist), _ptr(t_end), x0, nc, ctypes.byref(opts),
                                      _ptr(t), _ptr(G), cap, _ptr(nk), _ptr(st))
        check(rc, self._ctx, "sbr_learn_hetero")
        return dict(t=t, G=G, n_knots=nk, status=st)

    def hetero_point_paths(self, betas, dist, eta, t_end, u, p, kappa, lam, x0=1e-4, cap=65536) -> dict:
        """One heterogeneity equilibrium with learning knots t, group CDFs G [n, K], the
        per-group buffers, AW_total(t) and the per-group AW_OUT_k / AW_IN_k curves on the knots
        (aw_out / aw_in [K, n]) — what scripts/2_heterogeneity.jl plots."""
        betas = np.ascontiguousarray(betas, np.float64)
        dist = np.ascontiguousarray(dist, np.float64)
        K = len(dist)
        res = np.zeros(3)
        st = np.zeros(1, np.uint32)
        tin, tout = np.empty(K), np.empty(K)
        t, G, aw = np.empty(cap), np.empty(cap * K), np.empty(cap)
        awg = np.empty((2 * K, cap))
        nk = ctypes.c_int64()
        opts = _lib.default_opts(early_exit_nan_run=0, knot_capacity=16384)
        rc = self._L.sbr_hetero_point_paths(self._ctx, K, _ptr(betas), _ptr(dist), eta, t_end, x0, u, p, kappa, lam,
                                            ctypes.byref(opts), _ptr(res), _ptr(st), _ptr(tin), _ptr(tout), _ptr(t),
                                            _ptr(G), _ptr(aw), _ptr(awg), cap, ctypes.byref(nk))
        check(rc, self._ctx, "sbr_hetero_point_paths")
        n = nk.value
        return dict(xi=res[0], aw_max=res[1], tol=res[2], status=int(st[0]), tau_in_unc=tin, tau_out_unc=tout,
                    t=t[:n].copy(), G=G[:n * K].reshape(n, K).copy(), aw_total=aw[:n].copy(),
                    aw_out=awg[:K, :n].copy(), aw_in=awg[K:, :n].copy())

    def interest_point_paths(self, beta, eta, t_end, u, p, kappa, lam, r, delta, x0=1e-4, cap=65536) -> dict:
        """One interest-rate equilibrium with τ̄, HR(τ̄), V(τ̄) (saved on the HR grid) and
        AW_cum(τ̄) — what scripts/3_interest_rates.jl plots."""
        res = np.zeros(5)
        st = np.zeros(1, np.uint32)
        tau, hr, V, aw = np.empty(cap), np.empty(cap), np.empty(cap), np.empty(cap)
        nt, nv = ctypes.c_int64(), ctypes.c_int64()
        opts = _lib.default_opts(early_exit_nan_run=0)
        rc = self._L.sbr_interest_point_paths(self._ctx, beta, eta, t_end, x0, u, p, kappa, lam, r, delta,
                                              ctypes.byref(opts), _ptr(res), _ptr(st), _ptr(tau), _ptr(hr), _ptr(V),
                                              _ptr(aw), cap, ctypes.byref(nt), ctypes.byref(nv))
        check(rc, self._ctx, "sbr_interest_point_paths")
        k, m = nt.value, nv.value
        return dict(xi=res[0], tau_in_unc=res[1], tau_out_unc=res[2], aw_max=res[3], tol=res[4], status=int(st[0]),
                    hr_tau=tau[:k].copy(), hr=hr[:k].copy(), V=V[:m].copy(), aw_cum=aw[:k].copy())

    def sweep_interest_dev(self, beta, eta, t_end, u, p, kappa, lam, r, delta, x0, out: dict,
                           stream: int | None = None, max_iters: int = 100, knot_capacity: int = 65536):
        """Device-pointer interest sweep on torch tensors (enqueue only)."""
        nb, nu = beta.numel(), u.numel()
        soa = _lib.ResultSoA(*_out_ptrs(out, (*RESULT_FIELDS, "status", "iters"), nb * nu,
                                        required=(*RESULT_FIELDS, "status")))
        opts = _lib.default_opts(early_exit_nan_run=0, bisect_max_iters=max_iters, knot_capacity=knot_capacity)
        (rk,) = _out_ptrs(out, ("rk_steps",), nb * nu)
        rc = self._L.sbr_sweep_interest_dev(self._ctx, stream, _dptr(beta, "beta", _F64), _dptr(eta, "eta", _F64, nb),
                                            _dptr(t_end, "t_end", _F64, nb), x0, _dptr(u, "u", _F64), nb, nu, p,
                                            kappa, lam, r, delta, ctypes.byref(opts), ctypes.byref(soa), rk)
        check(rc, self._ctx, "sbr_sweep_interest_dev")

    def social_prof_read(self) -> list[int]:
        v = (ctypes.c_int64 * 8)()
        check(self._L.sbr_social_prof_read(self._ctx, v), self._ctx, "sbr_social_prof_read")
        return list(v)

    def social_overflow_stats(self) -> dict:
        """Last social sweep: points promoted into the 16x pool / re-run from scratch larger."""
        a, b = ctypes.c_int64(), ctypes.c_int64()
        check(self._L.sbr_social_overflow_stats(self._ctx, ctypes.byref(a), ctypes.byref(b)), self._ctx,
              "sbr_social_overflow_stats")
        return dict(promoted=a.value, rerun=b.value)

    def device_info(self) -> dict:
        a, b, c = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(self._L.sbr_device_info(self._ctx, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), self._ctx,
              "sbr_device_info")
        return dict(lds_bytes_per_block=a.value, lds_knot_capacity=b.value, cu_count=c.value)

    def host_phases(self) -> dict:
        """Phases (ms) of the last host-pointer sweep_baseline made with timing enabled; on an
        n-device context, of the last host-pointer sweep's fan-out (always recorded)."""
        v = (ctypes.c_double * 5)()
        check(self._L.sbr_host_phases(self._ctx, v), self._ctx, "sbr_host_phases")
        if self.n_gpus > 1 or self._multi:
            return dict(zip(("slowest_rank_sweep", "slowest_rank_d2h_pinned", "host_copy_or_gather", "unused",
                             "call"), list(v)))
        return dict(zip(("h2d", "kernels", "d2h", "host_copy_early_exit", "call"), list(v)))

    def chunk_timeline(self, stream: int | None = None) -> list:
        """[(learning end, equilibrium end)] in ms per column chunk of the last chunked single
        sweep made with timing enabled (sbr_chunk_timeline); [] otherwise."""
        n = ctypes.c_int32()
        v = (ctypes.c_double * 16)()
        check(self._L.sbr_chunk_timeline(self._ctx, stream, ctypes.byref(n), v), self._ctx, "sbr_chunk_timeline")
        return [(v[2 * k], v[2 * k + 1]) for k in range(n.value)]

    def last_schedule(self) -> int:
        """1 if the last single sweep took the per-column readiness schedule, 0 if chunked."""
        v = ctypes.c_int32()
        check(self._L.sbr_last_schedule(self._ctx, ctypes.byref(v)), self._ctx, "sbr_last_schedule")
        return v.value

    def timing_enable(self, on: bool = True):
        check(self._L.sbr_timing_enable(self._ctx, int(on)), self._ctx, "sbr_timing_enable")

    def timing_read(self, stream: int | None = None):
        """(learn_ms_total, equilibrium_ms_total, n_calls) since the last read."""
        a, b, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int32()
        check(self._L.sbr_timing_read(self._ctx, stream, ctypes.byref(a), ctypes.byref(b), ctypes.byref(n)),
              self._ctx, "sbr_timing_read")
        return a.value, b.value, n.value

    def learn_stats(self, n_beta: int) -> dict:
        out = {k: np.zeros(n_beta, np.int32) for k in ("n_knots", "n_tau", "n_accept", "n_reject")}
        out["status"] = np.zeros(n_beta, np.uint32)
        check(self._L.sbr_learn_stats(self._ctx, n_beta, *[_ptr(out[k]) for k in
                                                         ("n_knots", "n_tau", "n_accept", "n_reject", "status")]),
              self._ctx, "sbr_learn_stats")
        return out

    def hetero_learn_stats(self, n_col: int) -> dict:
        out = {k: np.zeros(n_col, np.int32) for k in ("n_knots", "n_tau", "n_accept", "n_reject")}
        out["status"] = np.zeros(n_col, np.uint32)
        check(self._L.sbr_hetero_learn_stats(self._ctx, n_col, *[_ptr(out[k]) for k in
                                                                ("n_knots", "n_tau", "n_accept", "n_reject",
                                                                 "status")]),
              self._ctx, "sbr_hetero_learn_stats")
        return out

    def selftest_fastpow(self, x, y):
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        out = np.empty(len(x))
        check(self._L.sbr_selftest_fastpow(self._ctx, _ptr(x), _ptr(y), len(x), _ptr(out)), self._ctx,
              "sbr_selftest_fastpow")
        return out

    def selftest_detmath(self, x, y):
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        n = len(x)
        e, l, pw = np.empty(n), np.empty(n), np.empty(n)
        rc = self._L.sbr_selftest_detmath(self._ctx, _ptr(x), _ptr(y), n, _ptr(e), _ptr(l), _ptr(pw))
        check(rc, self._ctx, "sbr_selftest_detmath")
        return e, l, pw


_default: Engine | None = None


def default_engine() -> Engine:
    global _default
    if _default is None:
        _default = Engine()
    return _default


# ---------------------------------------------------------------------------
# Interpolations.jl-like gridded linear interpolant (host side, for the
# plotting drop-in; the hot path never uses it).
# ---------------------------------------------------------------------------
class LinearInterpolation:
    """Gridded Linear with Throw() extrapolation: exact at knots, BoundsError
    (IndexError here) outside [knots[0], knots[-1]]."""

    def __init__(self, knots, values):
        self.knots = np.asarray(knots, np.float64)
        self.coefs = np.asarray(values, np.float64)

    def __call__(self, x):
        x = np.asarray(x, np.float64)
        if np.any(~((x >= self.knots[0]) & (x <= self.knots[-1]))):
            raise IndexError("BoundsError: interpolation outside the knot range")
        n = len(self.knots)
        j = np.clip(np.searchsorted(self.knots, x, side="right") - 1, 0, n - 2)
        t0, t1 = self.knots[j], self.knots[j + 1]
        d = (x - t0) / (t1 - t0)
        v = self.coefs[j] * (1.0 - d) + self.coefs[j + 1] * d
        return v if v.ndim else float(v)


@dataclass
class LearningResults:
    """learning.jl:74-81 (grid = knots of the adaptive ODE solution)."""

    params: LearningParameters
    learning_cdf: LinearInterpolation
    learning_pdf: LinearInterpolation
    grid: np.ndarray
    status: int = 0


@dataclass
class SolvedModel:
    """solver.jl:55-109 (fields + derived τ_IN/τ_OUT; HR as an interpolant)."""

    xi: float
    tau_bar_IN_UNC: float
    tau_bar_OUT_UNC: float
    HR: LinearInterpolation
    bankrun: bool
    model_params: tuple
    learning_results: LearningResults
    converged: bool
    tolerance: float
    status: int
    aw_cum: np.ndarray = field(repr=False, default=None)
    aw: dict | None = field(repr=False, default=None)
    # (AW_OUT, AW_IN, AW_max) from the engine (solve_equilibrium_baseline on the caller's knots)
    aw_paths: tuple | None = field(repr=False, default=None)

    @property
    def tau_IN(self):
        return max(self.xi - self.tau_bar_IN_UNC, 0.0) if self.xi == self.xi else float("nan")

    @property
    def tau_OUT(self):
        return max(self.xi - self.tau_bar_OUT_UNC, 0.0) if self.xi == self.xi else float("nan")


def solve_learning(lp: LearningParameters, engine: Engine | None = None, tol: float | None = None) -> LearningResults:
    """learning.jl:109-124 on the GPU (full tspan, like the reference); ``tol`` = the ODE's
    reltol = abstol (None: eps(), learning.jl:43)."""
    if lp.tspan[0] != 0.0:
        raise _lib.ArgumentError("the engine integrates from t = 0 (every reference call site does)")
    eng = engine or default_engine()
    (t, G, st), = eng.learn_baseline([lp.beta], [lp.tspan[1]], [lp.tspan[1]], lp.x0, stop_after_eta=False, tol=tol)
    g = (lp.beta * G) * (1.0 - G)
    return LearningResults(lp, LinearInterpolation(t, G), LinearInterpolation(t, g), t, st)


def solve_equilibrium_baseline(lr: LearningResults, econ: EconomicParameters,
                               engine: Engine | None = None, xi_guess: float | None = None) -> SolvedModel:
    """solver.jl:413-462 for one point on the GPU, on ``lr``'s own knots (no learning ODE: the
    scripts learn once per β and call this per u, 1_baseline.jl:169, 248), with the HR path and
    get_AW's three paths."""
    eng = engine or default_engine()
    lp = lr.params
    cdf = lr.learning_cdf
    r = eng.equilibrium_on_knots(cdf.knots, cdf.coefs, lp.beta, econ.eta, lp.tspan[1], econ.u, econ.p, econ.kappa,
                                 econ.lam, xi_guess=xi_guess)
    # the learning solve's own status bits, as a sweep point carries them (maxiters, stiff switch)
    st = int(r["status"][0]) | (lr.status & _LEARN_BITS)
    if st & _lib.SBR_OOB:
        raise IndexError("BoundsError: interpolation outside the knot range (solver.jl, Interpolations Throw())")
    bankrun = bool(st & _lib.SBR_RUN)
    sm = SolvedModel(float(r["xi"][0]), float(r["tau_in_unc"][0]), float(r["tau_out_unc"][0]),
                     LinearInterpolation(r["tau"], r["hr"]), bankrun, (lp, econ), lr, bool(st & _lib.SBR_CONVERGED),
                     float(r["tol"][0]), st, aw_cum=r["aw_cum"],
                     aw_paths=(r["aw_out"], r["aw_in"], float(r["aw_max"][0])))
    return sm


def solve_equilibrium_social_learning(model: ModelParameters, tol: float = 1e-4, max_iter: int = 250,
                                      engine: Engine | None = None) -> SolvedModel:
    """social_learning_solver.jl:63-263 for one ModelParameters on the GPU: tspan is
    overridden to (0, η) (:79); returns the last inner equilibrium like the reference
    (HR / AW paths are not materialised for the social path; ``status`` carries
    SBR_SOCIAL_NOT_CONVERGED and the fixed-point iteration count is ``fp_iters``)."""
    eng = engine or default_engine()
    lp, econ = model.learning, model.economic
    r = eng.sweep_social([lp.beta], econ.eta, [econ.u], econ.p, econ.kappa, econ.lam, x0=float(np.ravel(lp.x0)[0]),
                         tol=tol, max_iter=max_iter)
    st = int(r["status"][0, 0])
    lr = LearningResults(LearningParameters(lp.beta, (0.0, econ.eta), lp.x0), None, None, np.empty(0), st)
    sm = SolvedModel(float(r["xi"][0, 0]), float(r["tau_in_unc"][0, 0]), float(r["tau_out_unc"][0, 0]), None,
                     bool(st & _lib.SBR_RUN), (lr.params, econ), lr, bool(st & _lib.SBR_CONVERGED),
                     float(r["tol"][0, 0]), st)
    sm.fp_iters = int(r["fp_iters"][0, 0])
    if sm.bankrun:
        sm.aw = dict(AW_max=float(r["aw_max"][0, 0]))
    return sm


def get_AW_functions(result: SolvedModel):
    """solver.jl:553-576: AW_cum/AW_OUT/AW_IN interpolants on the HR grid and
    AW_max, or None when there is no run.  AW_OUT/AW_IN are rebuilt on the host
    from the GPU's ξ, τ̄ and G (plotting only)."""
    if result.aw is not None:
        return result.aw
    if not result.bankrun:
        return None
    tg = result.HR.knots
    if result.aw_paths is not None:  # the engine's get_AW paths and AW_max
        aw_out, aw_in, aw_max = result.aw_paths
        result.aw = dict(AW_cum=LinearInterpolation(tg, result.aw_cum), AW_OUT=LinearInterpolation(tg, aw_out),
                         AW_IN=LinearInterpolation(tg, aw_in), AW_max=aw_max)
        return result.aw
    cdf = result.learning_results.learning_cdf
    xi, tin, tout = result.xi, result.tau_bar_IN_UNC, result.tau_bar_OUT_UNC
    ic = xi if tin >= xi else tin
    oc = xi if tout > xi else tout
    a = (tg - xi) + ic
    b = (tg - xi) + oc
    aw_in = np.where(a >= 0, cdf(np.where(a > 0, a, 0.0)), 0.0)
    aw_out = np.where(b >= 0, cdf(np.where(b > 0, b, 0.0)), 0.0)
    result.aw = dict(AW_cum=LinearInterpolation(tg, result.aw_cum), AW_OUT=LinearInterpolation(tg, aw_out),
                     AW_IN=LinearInterpolation(tg, aw_in), AW_max=float(np.max(result.aw_cum)))
    return result.aw


@dataclass
class SolvedModelInterest(SolvedModel):
    """interest_rate_model.jl:200-245: SolvedModel plus the value function V
    (LinearInterpolation on the HR grid; None when r = 0)."""

    V: LinearInterpolation | None = field(repr=False, default=None)


def solve_equilibrium_interest(lr: LearningResults, econ: EconomicParametersInterest,
                               model: ModelParametersInterest | None = None,
                               engine: Engine | None = None) -> SolvedModelInterest:
    """interest_rate_solver.jl:51-150 for one point on the GPU: HR, the value function
    saved on the HR grid (r > 0), buffers on h − rV, compute_ξ, and the AW paths."""
    eng = engine or default_engine()
    lp = lr.params
    r = eng.interest_point_paths(lp.beta, econ.eta, lp.tspan[1], econ.u, econ.p, econ.kappa, econ.lam, econ.r,
                                 econ.delta, lp.x0)
    st = r["status"]
    V = LinearInterpolation(r["hr_tau"][:len(r["V"])], r["V"]) if econ.r > 0 and len(r["V"]) >= 2 else None
    return SolvedModelInterest(r["xi"], r["tau_in_unc"], r["tau_out_unc"], LinearInterpolation(r["hr_tau"], r["hr"]),
                               bool(st & _lib.SBR_RUN), (lp, econ) if model is None else model, lr,
                               bool(st & _lib.SBR_CONVERGED), r["tol"], st, aw_cum=r["aw_cum"], V=V)


def get_AW_functions_interest(result: SolvedModelInterest):
    """interest_rate_solver.jl:161-184: the baseline get_AW on the HR grid (None without a run)."""
    return get_AW_functions(result)


@dataclass
class SolvedModelHetero:
    """heterogeneity_model.jl SolvedModelHetero: ξ, the per-group buffers, the learning
    knots / group CDFs and AW_total on the knots (get_AW_functions_hetero!)."""

    xi: float
    tau_bar_IN_UNCs: np.ndarray
    tau_bar_OUT_UNCs: np.ndarray
    bankrun: bool
    converged: bool
    tolerance: float
    status: int
    t: np.ndarray = field(repr=False)
    G: np.ndarray = field(repr=False)
    AW_total: np.ndarray = field(repr=False)
    AW_max: float = float("nan")
    HRs: list = field(repr=False, default_factory=list)  # HR_k on the τ̄ grid (heterogeneity_solver.jl:255)
    learning_results: object = field(repr=False, default=None)
    # get_AW_hetero's per-group curves on the knots, from the engine (heterogeneity_solver.jl:335-362)
    AW_OUT_groups: np.ndarray = field(repr=False, default=None)  # [K, n]
    AW_IN_groups: np.ndarray = field(repr=False, default=None)   # [K, n]

    def get_AW_functions_hetero(self):
        """get_AW_functions_hetero! (heterogeneity_solver.jl:386-402): (AW_cum, AW_OUT_groups,
        AW_IN_groups, AW_groups, AW_max) as interpolants on the knots, None without a run.
        AW_groups = AW_OUT_k − AW_IN_k as get_AW_hetero forms them (:358)."""
        if not self.bankrun:
            return None
        t = self.t
        outs = [LinearInterpolation(t, self.AW_OUT_groups[k]) for k in range(len(self.AW_OUT_groups))]
        ins = [LinearInterpolation(t, self.AW_IN_groups[k]) for k in range(len(self.AW_IN_groups))]
        nets = [LinearInterpolation(t, self.AW_OUT_groups[k] - self.AW_IN_groups[k]) for k in range(len(outs))]
        return dict(AW_cum=LinearInterpolation(t, self.AW_total), AW_OUT_groups=outs, AW_IN_groups=ins,
                    AW_groups=nets, AW_max=self.AW_max)


@dataclass
class LearningResultsHetero:
    """heterogeneity_model.jl LearningResultsHetero: the shared knot grid and the K group CDFs
    (learning_cdfs[k] = LinearInterpolation(grid, G[:, k])) / PDFs of solve_SInetwork_hetero."""

    params: LearningParametersHetero
    learning_cdfs: list
    learning_pdfs: list
    grid: np.ndarray
    G: np.ndarray = field(repr=False)  # [n, K], the CDFs' values (knot-major, as libsbr takes them)
    status: int = 0


def solve_SInetwork_hetero(lp: LearningParametersHetero, engine: Engine | None = None) -> LearningResultsHetero:
    """heterogeneity_learning.jl:49-94 on the GPU (sbr_learn_hetero: the coupled
    AutoTsit5(Rosenbrock23()) solve at eps(), full tspan) with compute_pdf_hetero (:114-134):
    pdf_k = (1 − G_k)·β_k·ω, ω = Σ_j dist_j G_j (left fold)."""
    if lp.tspan[0] != 0.0:
        raise _lib.ArgumentError("the engine integrates from t = 0 (every reference call site does)")
    eng = engine or default_engine()
    betas, dist = np.array(lp.betas), np.array(lp.dist)
    K = len(dist)
    r = eng.learn_hetero(betas[None, :], dist, lp.tspan[1], lp.x0, cap=16384)
    n = int(r["n_knots"][0])
    t, G = r["t"][0, :n].copy(), np.ascontiguousarray(r["G"][0, :n, :])
    w = dist[0] * G[:, 0]
    for j in range(1, K):
        w = w + dist[j] * G[:, j]
    cdfs = [LinearInterpolation(t, G[:, k].copy()) for k in range(K)]
    pdfs = [LinearInterpolation(t, ((1.0 - G[:, k]) * betas[k]) * w) for k in range(K)]
    return LearningResultsHetero(lp, cdfs, pdfs, t, G, int(r["status"][0]))


def solve_equilibrium_hetero(lr_or_model, econ: EconomicParameters | None = None,
                             engine: Engine | None = None) -> SolvedModelHetero:
    """heterogeneity_solver.jl:241-293 + get_AW_functions_hetero! (:386) for one point:
    ``solve_equilibrium_hetero(lr_hetero, econ)`` solves on the LearningResultsHetero's own
    knots and group CDFs (sbr_hetero_equilibrium_on_knots; no learning ODE); the HRs are the
    engine's HR_k on the τ̄ grid.  ``solve_equilibrium_hetero(model)`` (ModelParametersHetero)
    learns first."""
    eng = engine or default_engine()
    if isinstance(lr_or_model, ModelParametersHetero):
        lr, econ = solve_SInetwork_hetero(lr_or_model.learning, eng), lr_or_model.economic
    else:
        lr = lr_or_model
    lp = lr.params
    r = eng.hetero_equilibrium_on_knots(lr.grid, lr.G, np.array(lp.betas), np.array(lp.dist), econ.eta, lp.tspan[1],
                                        econ.u, econ.p, econ.kappa, econ.lam)
    st = int(r["status"][0]) | (lr.status & _LEARN_BITS)
    tau = np.append(lr.grid[lr.grid <= econ.eta], econ.eta)[:r["n_tau"]]
    HRs = [LinearInterpolation(tau, r["hr"][k]) for k in range(len(lp.dist))] if r["n_tau"] else []
    return SolvedModelHetero(float(r["xi"][0]), r["tau_in_unc"][0], r["tau_out_unc"][0], bool(st & _lib.SBR_RUN),
                             bool(st & _lib.SBR_CONVERGED), float(r["tol"][0]), st, lr.grid, lr.G, r["aw_total"],
                             float(r["aw_max"][0]), HRs, lr, r["aw_out"], r["aw_in"])
