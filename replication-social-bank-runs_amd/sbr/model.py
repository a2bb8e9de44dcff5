"""Parameter records — mirror of src/baseline/model.jl and
src/extensions/heterogeneity/heterogeneity_model.jl.

Same field names, same defaults, same validation (raising ArgumentError),
and — importantly for drop-in parity — the same copy-modify semantics:
``ModelParameters(base, beta=...)`` carries η and tspan over from ``base``
(model.jl:189-211) instead of re-deriving η = η_bar/β; that carry-over is what
the Fig 3bis and Fig 5 results depend on.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ._lib import ArgumentError

__all__ = [
    "LearningParameters",
    "EconomicParameters",
    "ModelParameters",
    "LearningParametersHetero",
    "ModelParametersHetero",
]


@dataclass(frozen=True)
class LearningParameters:
    """model.jl:24-39"""

    beta: float
    tspan: tuple[float, float]
    x0: float

    def __post_init__(self):
        b, ts, x0 = self.beta, self.tspan, self.x0
        if not b > 0:
            raise ArgumentError(f"Communication speed β must be positive, got β = {b}")
        if len(ts) != 2:
            raise ArgumentError("Time span tspan must be a tuple of length 2")
        if not ts[0] >= 0:
            raise ArgumentError(f"Start time must be non-negative, got tspan[1] = {ts[0]}")
        if not ts[1] > ts[0]:
            raise ArgumentError(f"End time must be greater than start time, got tspan = {ts}")
        if not x0 >= 0:
            raise ArgumentError(f"Initial condition x0 must be non-negative, got x0 = {x0}")
        object.__setattr__(self, "tspan", (float(ts[0]), float(ts[1])))


@dataclass(frozen=True)
class EconomicParameters:
    """model.jl:61-80"""

    u: float
    p: float
    kappa: float
    lam: float
    eta_bar: float
    eta: float

    def __post_init__(self):
        if not self.u >= 0:
            raise ArgumentError(f"Utility flow u must be non-negative, got u = {self.u}")
        if not 0 <= self.p <= 1:
            raise ArgumentError(f"Prior probability p must be in [0,1], got p = {self.p}")
        if not 0 < self.kappa < 1:
            raise ArgumentError(f"Solvency threshold κ must be in (0,1), got κ = {self.kappa}")
        if not self.lam > 0:
            raise ArgumentError(f"Exponential rate λ must be positive, got λ = {self.lam}")
        if not self.eta_bar > 0:
            raise ArgumentError(f"Raw awareness window η_bar must be positive, got η_bar = {self.eta_bar}")
        if not self.eta > 0:
            raise ArgumentError(f"Normalized awareness window η must be positive, got η = {self.eta}")


@dataclass(frozen=True)
class ModelParameters:
    """model.jl:109-116 plus the keyword (150-176) and copy-modify (189-211)
    constructors, exposed as ``ModelParameters.make(...)`` and
    ``ModelParameters.modify(base, ...)`` (``ModelParameters(base, **kw)`` in
    Julia)."""

    learning: LearningParameters
    economic: EconomicParameters

    @staticmethod
    def make(beta=1.0, eta=None, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01, tspan=None, x0=0.0001):
        if eta is None:
            eta = _fdiv(eta_bar, beta)  # Float64 division: β = 0 gives Inf, then ArgumentError below
        if tspan is None:
            tspan = (0.0, 2 * eta)
        return ModelParameters(LearningParameters(beta, tspan, x0), EconomicParameters(u, p, kappa, lam, eta_bar, eta))

    @staticmethod
    def modify(base: "ModelParameters", **kw) -> "ModelParameters":
        cur = dict(
            beta=base.learning.beta, eta=base.economic.eta, eta_bar=base.economic.eta_bar, u=base.economic.u,
            p=base.economic.p, kappa=base.economic.kappa, lam=base.economic.lam, tspan=base.learning.tspan,
            x0=base.learning.x0,
        )
        unknown = set(kw) - set(cur)
        if unknown:
            raise TypeError(f"unknown parameters {sorted(unknown)}")
        cur.update(kw)
        return ModelParameters.make(**cur)


@dataclass(frozen=True)
class LearningParametersHetero:
    """heterogeneity_model.jl:25-45"""

    betas: tuple[float, ...]
    dist: tuple[float, ...]
    tspan: tuple[float, float]
    x0: float

    def __post_init__(self):
        betas, dist = tuple(float(b) for b in self.betas), tuple(float(d) for d in self.dist)
        if len(betas) < 1:
            raise ArgumentError(f"Must have at least one group, got {len(betas)} groups")
        if len(dist) != len(betas):
            raise ArgumentError(f"Distribution length {len(dist)} must match βs length {len(betas)}")
        if not all(b > 0 for b in betas):
            raise ArgumentError("All learning rates βs must be positive")
        if not all(d >= 0 for d in dist):
            raise ArgumentError("All distribution weights must be non-negative")
        if not abs(_jl_sum(dist) - 1.0) < 1e-10:
            raise ArgumentError(f"Distribution must sum to 1, got sum = {sum(dist)}")
        ts = self.tspan
        if len(ts) != 2:
            raise ArgumentError("Time span must be a tuple of length 2")
        if not ts[0] >= 0:
            raise ArgumentError("Start time must be non-negative")
        if not ts[1] > ts[0]:
            raise ArgumentError("End time must be greater than start time")
        if not self.x0 >= 0:
            raise ArgumentError("Initial condition must be non-negative")
        object.__setattr__(self, "betas", betas)
        object.__setattr__(self, "dist", dist)
        object.__setattr__(self, "tspan", (float(ts[0]), float(ts[1])))


def _fdiv(a, b) -> float:
    """IEEE division as in Julia (x/0.0 = ±Inf, 0/0 = NaN) instead of ZeroDivisionError."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return float(np.float64(a) / np.float64(b))


def _jl_sum(xs):
    """Julia's sum over a Vector{Float64} (pairwise for n > 16; plain
    left-to-right below, which is every K used here)."""
    s = 0.0
    for x in xs:
        s += x
    return s


@dataclass(frozen=True)
class ModelParametersHetero:
    """heterogeneity_model.jl:75-144 (η = η_bar / Σ dist·βs) and the
    copy-modify constructor 157-179 (re-derives η, carries tspan)."""

    learning: LearningParametersHetero
    economic: EconomicParameters

    @staticmethod
    def make(betas, dist, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01, tspan=None, x0=0.0001):
        betas, dist = tuple(float(b) for b in betas), tuple(float(d) for d in dist)
        if len(betas) < 1:
            raise ArgumentError("βs cannot be empty")
        if len(dist) != len(betas):
            raise ArgumentError("dist must have same length as βs")
        beta_ave = _jl_sum([d * b for d, b in zip(dist, betas)])
        eta = _fdiv(eta_bar, beta_ave)
        if tspan is None:
            tspan = (0.0, 2 * eta)
        return ModelParametersHetero(LearningParametersHetero(betas, dist, tspan, x0),
                                     EconomicParameters(u, p, kappa, lam, eta_bar, eta))

    @staticmethod
    def modify(base: "ModelParametersHetero", **kw) -> "ModelParametersHetero":
        cur = dict(betas=base.learning.betas, dist=base.learning.dist, eta_bar=base.economic.eta_bar,
                   u=base.economic.u, p=base.economic.p, kappa=base.economic.kappa, lam=base.economic.lam,
                   tspan=base.learning.tspan, x0=base.learning.x0)
        cur.update(kw)
        return ModelParametersHetero.make(**cur)


@dataclass(frozen=True)
class EconomicParametersInterest:
    """interest_rate_model.jl:25-54: the baseline economic parameters plus the
    interest rate r and deposit maturity rate δ (0 ≤ r < δ)."""

    u: float
    p: float
    kappa: float
    lam: float
    eta_bar: float
    eta: float
    r: float
    delta: float

    def __post_init__(self):
        EconomicParameters(self.u, self.p, self.kappa, self.lam, self.eta_bar, self.eta)  # shared checks (:40-45)
        if not self.r >= 0:
            raise ArgumentError(f"Interest rate r must be non-negative, got r = {self.r}")
        if not self.delta > 0:
            raise ArgumentError(f"Recovery rate δ must be positive, got δ = {self.delta}")
        if not self.r < self.delta:
            raise ArgumentError("Interest rate r must be less than recovery rate δ for convergence, "
                                f"got r = {self.r}, δ = {self.delta}")


@dataclass(frozen=True)
class ModelParametersInterest:
    """interest_rate_model.jl:82-92 with the keyword constructor (:120-148; η = η_bar/β,
    tspan = (0, 2η), r = 0, δ = 0.1 defaults) and the copy-modify one (:161-185)."""

    learning: LearningParameters
    economic: EconomicParametersInterest

    @staticmethod
    def make(beta=1.0, eta=None, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01, r=0.0, delta=0.1, tspan=None,
             x0=0.0001):
        if eta is None:
            eta = _fdiv(eta_bar, beta)
        if tspan is None:
            tspan = (0.0, 2 * eta)
        return ModelParametersInterest(LearningParameters(beta, tspan, x0),
                                       EconomicParametersInterest(u, p, kappa, lam, eta_bar, eta, r, delta))

    @staticmethod
    def modify(base: "ModelParametersInterest", **kw) -> "ModelParametersInterest":
        e = base.economic
        cur = dict(beta=base.learning.beta, eta=e.eta, eta_bar=e.eta_bar, u=e.u, p=e.p, kappa=e.kappa, lam=e.lam,
                   r=e.r, delta=e.delta, tspan=base.learning.tspan, x0=base.learning.x0)
        unknown = set(kw) - set(cur)
        if unknown:
            raise TypeError(f"unknown parameters {sorted(unknown)}")
        cur.update(kw)
        return ModelParametersInterest.make(**cur)
