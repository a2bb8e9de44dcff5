"""Sweep persistence and figure regeneration, on
oracle results (no GPU needed: the format is the engine's result dict)."""
import numpy as np

import sbr
from sbr import figures
from sbr import io as sio


def _small(oracle):
    g = sbr.fig5_grid(12, n_u=15)
    r = oracle.sweep_baseline(g.beta, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0)
    return g, r


def test_save_load_roundtrip(tmp_path, oracle):
    g, r = _small(oracle)
    p = sio.save_sweep(tmp_path / "fig5.npz", r, beta=g.beta, u=g.u, eta=g.eta, t_end=g.t_end,
                       params=dict(p=g.p, kappa=g.kappa, lam=g.lam, x0=g.x0), workload=g.name)
    arrays, meta = sio.load_sweep(p)
    for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol"):
        assert np.array_equal(arrays[k], r[k], equal_nan=True), k
    assert np.array_equal(arrays["status"], r["status"])
    assert arrays["status"].dtype == np.uint32
    assert meta["workload"] == g.name and meta["params"]["kappa"] == g.kappa
    assert meta["status_bits"]["SBR_RUN"] == sbr.STATUS["SBR_RUN"]
    assert sio.max_aw_matrix(arrays).shape == (len(g.u), len(g.beta))


def test_figures_render(tmp_path, oracle):
    g, r = _small(oracle)
    arrays, _ = sio.load_sweep(sio.save_sweep(tmp_path / "s.npz", r, beta=g.beta, u=g.u))
    a = figures.heatmap_fig5(arrays, tmp_path / "heat.png")
    b = figures.comparative_statics_u(arrays, tmp_path / "cs.png")
    assert a.stat().st_size > 1000 and b.stat().st_size > 1000
