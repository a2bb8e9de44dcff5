"""Parameter grids of the reference's sweeps and of the benchmark configs.

``julia_range(a, b, n)`` restates Julia's ``range(a, b, length=n)`` for
Float64 endpoints (Base._linspace via TwicePrecision): when both endpoints
are short decimals Julia interpolates the exact rationals they denote, so
element k is the correctly rounded value of a + k (b − a)/(n − 1) computed
in exact arithmetic — which is what ``fractions.Fraction`` gives here.
"""
from __future__ import annotations

from fractions import Fraction
from math import gcd

import numpy as np

__all__ = ["julia_range", "fig4_grid", "fig5_grid", "BaselineGrid"]


_MAXINTFLOAT32 = 16777216  # maxintfloat(narrow(Float64)) = maxintfloat(Float32)
_MAXINTFLOAT64 = 9007199254740992


def _julia_rat(x: float):
    """Base.rat (range.jl): continued-fraction rational (a, b) with a/b == x in
    Float64, bounded by maxintfloat(Float32); (c, d) of the last convergent
    within the bound otherwise."""
    y = float(x)
    a = d = 1
    b = c = 0
    m = _MAXINTFLOAT32
    while abs(y) <= m:
        f = int(y)  # trunc
        y -= f
        a, c = f * a + c, a
        b, d = f * b + d, b
        if max(abs(a), abs(b)) > m:
            return c, d
        if float(a) / float(b) == x:
            break
        if y == 0.0:
            break
        y = 1.0 / y
    return a, b


def _endpoints(a, b):
    """Exact rationals Julia's _linspace(start, stop, len) interpolates between:
    the Base.rat representations when both pass its round-trip checks (short
    decimals like 0.001 -> 1/1000, 100/3 for 33.333333333333336), else the
    binary64 values themselves (the TwicePrecision fallback)."""
    fa, fb = float(Fraction(a)) if isinstance(a, str) else float(a), float(Fraction(b)) if isinstance(b, str) else float(b)
    an, ad = _julia_rat(fa)
    bn, bd = _julia_rat(fb)
    if ad != 0 and bd != 0:
        den = ad * bd // gcd(ad, bd)
        if den != 0 and abs(den * fa) <= _MAXINTFLOAT64 and abs(den * fb) <= _MAXINTFLOAT64:
            sn, en = round(den * fa), round(den * fb)
            if sn / den == fa and en / den == fb:
                return Fraction(sn, den), Fraction(en, den)
    return Fraction(fa), Fraction(fb)


def julia_range(a, b, n: int) -> np.ndarray:
    """range(a, b, length=n) for Float64 endpoints (elements correctly rounded
    from Julia's exact rational endpoints; TwicePrecision agrees to the ulp)."""
    if n == 1:
        return np.array([float(Fraction(a)) if isinstance(a, str) else float(a)])
    A, B = _endpoints(a, b)
    step = (B - A) / (n - 1)
    return np.array([float(A + step * k) for k in range(n)], dtype=np.float64)


class BaselineGrid:
    """β columns × u rows with per-β η and t_end (the copy-modify carry-over)."""

    def __init__(self, beta, u, eta, t_end, p=0.5, kappa=0.6, lam=0.01, x0=1e-4, name=""):
        self.beta = np.ascontiguousarray(beta, np.float64)
        self.u = np.ascontiguousarray(u, np.float64)
        self.eta = np.ascontiguousarray(np.broadcast_to(eta, self.beta.shape), np.float64)
        self.t_end = np.ascontiguousarray(np.broadcast_to(t_end, self.beta.shape), np.float64)
        self.p, self.kappa, self.lam, self.x0 = float(p), float(kappa), float(lam), float(x0)
        self.name = name

    @property
    def shape(self):
        return (len(self.beta), len(self.u))

    @property
    def n_points(self):
        return len(self.beta) * len(self.u)

    def subset(self, beta_idx) -> "BaselineGrid":
        return BaselineGrid(self.beta[beta_idx], self.u, self.eta[beta_idx], self.t_end[beta_idx], self.p,
                            self.kappa, self.lam, self.x0, self.name)


def fig4_grid(n: int = 5000) -> BaselineGrid:
    """scripts/1_baseline.jl:137 — u = range(0.001, 0.2, 5000) at β = 1 (m_base: η = 15, tspan = (0, 30))."""
    return BaselineGrid([1.0], julia_range("0.001", "0.2", n), 15.0, 30.0, name=f"fig4_u{n}")


def fig5_grid(n: int = 500, n_u: int | None = None) -> BaselineGrid:
    """scripts/1_baseline.jl:210-212 — ave_meeting_time = range(1e-4, 1, n), β = 1 ./ amt,
    u = range(0.001, 1, n); every β keeps m_base's η = 15 and tspan = (0, 30)
    (copy-modify carry-over, model.jl:189-211).  n = 2048 is benchmark config 3."""
    amt = julia_range("0.0001", "1", n)
    beta = 1.0 / amt
    u = julia_range("0.001", "1", n if n_u is None else n_u)
    return BaselineGrid(beta, u, 15.0, 30.0, name=f"fig5_{n}x{n if n_u is None else n_u}")


def _jl_sum(xs) -> float:
    s = 0.0
    for x in xs:
        s += x
    return s


class HeteroGrid:
    """K-group heterogeneity sweep: columns of group rates × u rows.  η is
    re-derived per column (η_bar / Σ dist·βs, heterogeneity_model.jl:131-132),
    tspan is carried from the base model (copy-modify, :157-179)."""

    def __init__(self, betas, dist, u, eta_bar=30.0, t_end=None, p=0.9, kappa=0.3, lam=0.1, x0=1e-4, name=""):
        self.betas = np.ascontiguousarray(np.atleast_2d(betas), np.float64)
        self.dist = np.ascontiguousarray(dist, np.float64)
        self.u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
        self.eta = np.array([eta_bar / _jl_sum(self.dist * b) for b in self.betas])
        if t_end is None:
            t_end = 2 * self.eta
        self.t_end = np.ascontiguousarray(np.broadcast_to(t_end, self.eta.shape), np.float64)
        self.p, self.kappa, self.lam, self.x0 = float(p), float(kappa), float(lam), float(x0)
        self.name = name

    @property
    def K(self):
        return self.betas.shape[1]

    @property
    def shape(self):
        return (self.betas.shape[0], len(self.u))

    @property
    def n_points(self):
        return self.shape[0] * self.shape[1]

    def subset(self, idx) -> "HeteroGrid":
        g = HeteroGrid.__new__(HeteroGrid)
        g.__dict__.update(self.__dict__)
        g.betas, g.eta, g.t_end = self.betas[idx], self.eta[idx], self.t_end[idx]
        return g


def hetero_script_grid() -> HeteroGrid:
    """scripts/2_heterogeneity.jl:38-49: βs = [0.125, 12.5], dist = [0.9, 0.1], η_bar = 30,
    u = 0.1, p = 0.9, κ = 0.3, λ = 0.1 (tspan = (0, 2η))."""
    return HeteroGrid([[0.125, 12.5]], [0.9, 0.1], [0.1], name="hetero_script")


def hetero_config4(n_s: int = 1024, n_u: int = 1024, K: int = 8) -> HeteroGrid:
    """BASELINE config 4 (concretised in SURVEY.md §8(d)): βs_k = s·0.125·100^((k−1)/(K−1))
    spanning Fig 9's 0.125…12.5 at s = 1, dist_k = 1/K, s = 1 ./ range(1e-3, 1, n_s),
    u = range(0.001, 1, n_u), η_bar = 30, p = 0.9, κ = 0.3, λ = 0.1; η re-derived per
    column, tspan carried from s = 1."""
    base = np.array([0.125 * 100.0 ** (k / (K - 1)) for k in range(K)]) if K > 1 else np.array([0.125])
    dist = np.full(K, 1.0 / K)
    s = 1.0 / julia_range("0.001", "1", n_s)
    betas = s[:, None] * base[None, :]
    t_end = 2 * 30.0 / _jl_sum(dist * base)
    return HeteroGrid(betas, dist, julia_range("0.001", "1", n_u), 30.0, t_end, name=f"hetero_K{K}_{n_s}x{n_u}")
