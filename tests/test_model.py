"""Host logic: parameter records (model.jl / heterogeneity_model.jl) and grids."""
import numpy as np
import pytest

import sbr
from sbr import ArgumentError, ModelParameters, ModelParametersHetero


def test_keyword_defaults():
    m = ModelParameters.make()  # model.jl:150-176
    assert m.learning.beta == 1.0 and m.learning.tspan == (0.0, 30.0) and m.learning.x0 == 1e-4
    e = m.economic
    assert (e.u, e.p, e.kappa, e.lam, e.eta_bar, e.eta) == (0.1, 0.5, 0.6, 0.01, 15.0, 15.0)


def test_copy_modify_carries_eta_and_tspan():
    """model.jl:189-211: ModelParameters(m_base; β=3) keeps η = 15 and tspan = (0, 30)."""
    base = ModelParameters.make(beta=1.0, eta_bar=15.0)
    fast = ModelParameters.modify(base, beta=3.0)
    assert fast.learning.beta == 3.0
    assert fast.economic.eta == 15.0 and fast.learning.tspan == (0.0, 30.0)
    fresh = ModelParameters.make(beta=3.0, eta_bar=15.0)
    assert fresh.economic.eta == 5.0 and fresh.learning.tspan == (0.0, 10.0)


@pytest.mark.parametrize("kw", [dict(beta=0.0), dict(beta=-1.0), dict(u=-0.1), dict(p=1.5), dict(kappa=0.0),
                                dict(kappa=1.0), dict(lam=0.0), dict(eta_bar=0.0), dict(x0=-1e-4),
                                dict(tspan=(1.0, 0.5)), dict(tspan=(-1.0, 2.0))])
def test_validation_raises_argument_error(kw):
    with pytest.raises(ArgumentError):
        ModelParameters.make(**kw)


def test_hetero_eta_and_copy_modify():
    """heterogeneity_model.jl:131-136 (η = η_bar/Σ dist β) and 157-179 (η re-derived, tspan carried)."""
    m = ModelParametersHetero.make([0.125, 12.5], [0.9, 0.1], eta_bar=30.0, u=0.1, p=0.9, kappa=0.3, lam=0.1)
    beta_ave = 0.9 * 0.125 + 0.1 * 12.5
    assert m.economic.eta == 30.0 / beta_ave
    assert m.learning.tspan == (0.0, 2 * 30.0 / beta_ave)
    m2 = ModelParametersHetero.modify(m, betas=[0.25, 25.0])
    assert m2.economic.eta == 30.0 / (0.9 * 0.25 + 0.1 * 25.0)
    assert m2.learning.tspan == m.learning.tspan
    with pytest.raises(ArgumentError):
        ModelParametersHetero.make([1.0, 2.0], [0.5, 0.6])
    with pytest.raises(ArgumentError):
        ModelParametersHetero.make([1.0, -2.0], [0.5, 0.5])


def test_julia_range_is_exact_decimal_interpolation():
    r = sbr.julia_range("0.001", "0.2", 5000)
    assert r[0] == 0.001 and r[-1] == 0.2 and len(r) == 5000
    # element 2718 (1-based) — the Fig 4 boundary point
    assert r[2717] == float(__import__("fractions").Fraction(1, 1000) + __import__("fractions").Fraction(199, 1000) * 2717 / 4999)
    g = sbr.fig5_grid(500)
    assert g.beta[0] == 1e4 and g.beta[-1] == 1.0 and g.u[-1] == 1.0
    assert np.all(np.diff(g.beta) < 0)


def test_interest_parameters_mirror_reference_checks():
    """interest_rate_model.jl:38-54, 120-185: defaults, η = η_bar/β, tspan = (0, 2η),
    the 0 ≤ r < δ checks, and copy-modify carrying η / tspan."""
    m = sbr.ModelParametersInterest.make(beta=1.0, eta_bar=15.0, u=0.0, r=0.06, delta=0.1)
    assert m.economic.eta == 15.0 and m.learning.tspan == (0.0, 30.0)
    assert (m.economic.r, m.economic.delta) == (0.06, 0.1)
    d = sbr.ModelParametersInterest.make()
    assert (d.economic.r, d.economic.delta, d.economic.u) == (0.0, 0.1, 0.1)
    for kw in (dict(r=-0.01), dict(delta=0.0), dict(r=0.1, delta=0.1), dict(kappa=1.0), dict(u=-1.0)):
        with pytest.raises(sbr.ArgumentError):
            sbr.ModelParametersInterest.make(**kw)
    m2 = sbr.ModelParametersInterest.modify(m, beta=2.0)
    assert m2.economic.eta == 15.0 and m2.learning.tspan == (0.0, 30.0)  # carried, as in the reference
    with pytest.raises(TypeError):
        sbr.ModelParametersInterest.modify(m, gamma=1.0)


def test_host_result_views_checks_caller_arrays():
    """sweep_baseline(out=...) hands the caller's arrays to the C ABI only when every field has
    the dtype, size and layout the call writes (engine.host_result_views)."""
    from sbr.engine import RESULT_FIELDS, host_result_views
    n = 12
    out = {k: np.zeros((3, 4)) for k in RESULT_FIELDS}
    out["status"] = np.zeros(n, np.uint32)
    v = host_result_views(out, n)
    assert v["iters"] is None and v["xi"].shape == (n,) and np.shares_memory(v["xi"], out["xi"])
    out["iters"] = np.zeros(n, np.int32)
    assert host_result_views(out, n)["iters"].base is out["iters"] or np.shares_memory(
        host_result_views(out, n)["iters"], out["iters"])
    for bad in (dict(out, status=np.zeros(n, np.int32)), dict(out, xi=np.zeros(n + 1)),
                dict(out, tol=np.zeros((4, 6))[:, ::2]), dict(out, aw_max=None),
                dict(out, iters=np.zeros(n, np.int64))):
        with pytest.raises(ArgumentError):
            host_result_views(bad, n)
