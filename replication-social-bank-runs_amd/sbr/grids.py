"""Parameter grids of the reference's sweeps and of the benchmark configs.

``julia_range(a, b, n)`` restates Julia's ``range(a, b, length=n)`` for
Float64 endpoints (Base._linspace via TwicePrecision): when both endpoints
are short decimals Julia interpolates the exact rationals they denote, so
element k is the correctly rounded value of a + k (b − a)/(n − 1) computed
in exact arithmetic — which is what ``fractions.Fraction`` gives here.
"""
from __future__ import annotations

from fractions import Fraction

import numpy as np

__all__ = ["julia_range", "fig4_grid", "fig5_grid", "BaselineGrid"]


def _rat(x) -> Fraction:
    if isinstance(x, str):
        return Fraction(x)
    return Fraction(repr(float(x)))


def julia_range(a, b, n: int) -> np.ndarray:
    if n == 1:
        return np.array([float(_rat(a))])
    A, B = _rat(a), _rat(b)
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
