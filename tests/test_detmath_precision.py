"""Accuracy pin of the shared deterministic math (include/sbr_detmath.h), which the oracle and
every device kernel compile: sbr_exp / sbr_log against mpmath at 60 significant digits on the
argument ranges the path uses.  Julia's table-driven Base.exp / Base.log are correctly rounded
to within 1 ulp too, so "≤ 1 ulp from the exact value" bounds the distance to the reference's
own results.  The device's bit-equality with the host is a separate GPU test
(test_detmath_host_device_bitwise).

Ranges:
  exp(λτ̄) of hazard_rate (solver.jl:168,181): λ up to 0.25 (the social script), τ̄ ≤ η ≤ 40
      → [0, 10]; the initial-dt heuristic's 10^(−(2 + log10 d)/6) → exp over [−50, 12];
  log of the initial-dt norms d (ode_determine_initdt) → [1e-30, 1e10] and [0.5, 2].
"""
import numpy as np
import pytest

mpmath = pytest.importorskip("mpmath")

N = 12000  # ≥ 10^4 arguments per function


def ulp_errors(x, got, fn):
    mpmath.mp.dps = 60
    err = np.empty(len(x))
    for i, (xi, gi) in enumerate(zip(x, got)):
        exact = fn(mpmath.mpf(float(xi)))
        ref = float(exact)  # the correctly rounded double
        ulp = float(np.spacing(abs(ref)))
        err[i] = abs(float(mpmath.mpf(float(gi)) - exact)) / ulp
    return err


def test_sbr_exp_within_one_ulp(oracle):
    rng = np.random.default_rng(7)
    x = np.concatenate([rng.uniform(0.0, 10.0, N // 2), rng.uniform(-50.0, 12.0, N // 2)])
    e, _, _ = oracle.detmath(x, np.zeros_like(x))
    err = ulp_errors(x, e, mpmath.exp)
    assert err.max() <= 1.0, float(err.max())
    frac = float((err > 0.5).mean())
    print(f"sbr_exp: max {err.max():.3f} ulp, {100 * frac:.1f}% of {len(x)} above 0.5 ulp")
    assert frac < 0.25


def test_sbr_log_within_one_ulp(oracle):
    rng = np.random.default_rng(8)
    x = np.concatenate([10.0 ** rng.uniform(-30.0, 10.0, N // 2), rng.uniform(0.5, 2.0, N // 2)])
    _, l, _ = oracle.detmath(x, np.zeros_like(x))
    err = ulp_errors(x, l, mpmath.log)
    assert err.max() <= 1.0, float(err.max())
    frac = float((err > 0.5).mean())
    print(f"sbr_log: max {err.max():.3f} ulp, {100 * frac:.1f}% of {len(x)} above 0.5 ulp")
    assert frac < 0.25
