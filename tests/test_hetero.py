"""Heterogeneity extension (src/extensions/heterogeneity/): oracle pinned to
the committed figure, GPU kernels bit-identical to the oracle."""
import numpy as np
import pytest

import sbr
from golden_util import interp


def _hetero_oracle(oracle, g):
    return oracle.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0)


def test_hetero_script_figure(oracle, golden):
    """scripts/2_heterogeneity.jl: ξ (vline; the x tick step must be one of GR's
    nice steps and exactly one matches), AW_max and the AW curves on
    range(0, 2ξ, 1000) (aggregate_withdrawals_hetero.pdf)."""
    gold = golden("hetero.json")
    g = sbr.hetero_script_grid()
    r = _hetero_oracle(oracle, g)
    assert r["status"][0, 0] & sbr.STATUS["SBR_RUN"]
    xi = r["xi"][0, 0]
    span = gold["x_last"] - gold["x_first"]
    cands = [step / gold["tick_spacing_px"] * span / 2 for step in (1, 2, 2.5, 5, 10)]
    prec = 0.02 / span * 2 * max(cands)
    hits = [c for c in cands if abs(c - xi) <= prec]
    assert len(hits) == 1, (xi, cands)
    # AW_total(t) on t = range(0, 2ξ, 1000): rebuild the path on the learning grid
    t, G, _ = oracle.learn_hetero(g.betas[0], g.dist, g.t_end[0])
    tin, tout = r["tau_in_unc"][0, 0], r["tau_out_unc"][0, 0]
    ts = np.linspace(0.0, 2 * xi, 1000)
    cum = np.zeros(len(t))
    groups = []
    for k in range(g.K):
        ic, oc = min(tin[k], xi), min(tout[k], xi)
        a, b = (t - xi) + ic, (t - xi) + oc
        awin = np.where(a >= 0, interp(t, G[:, k], np.where(a > 0, a, 0.0)), 0.0)
        awout = np.where(b >= 0, interp(t, G[:, k], np.where(b > 0, b, 0.0)), 0.0)
        cum = cum + g.dist[k] * (awout - awin)
        groups.append(awout - awin)
    assert abs(r["aw_max"][0, 0] - np.max(cum)) < 1e-15
    tol = 2 * gold["aw_precision"] + 3e-4  # plus the ξ uncertainty of the x map
    assert np.max(np.abs(interp(t, cum, ts) - np.array(gold["aw_total"]))) < tol
    assert np.max(np.abs(interp(t, groups[0], ts) - np.array(gold["aw_group1"]))) < tol
    assert np.max(np.abs(interp(t, groups[1], ts) - np.array(gold["aw_group2"]))) < tol


def test_hetero_k1_reduces_to_baseline_semantics(oracle):
    """K = 1, dist = [1]: the coupled ODE is the logistic (ω = G); the hetero
    solver differs from the baseline only where the reference code differs
    (bracket [0, 2τ̄_OUT], tol 1e-12, explicit-grid η, AW on the full grid)."""
    g = sbr.HeteroGrid([[1.0]], [1.0], sbr.julia_range("0.001", "0.2", 40), eta_bar=15.0, t_end=30.0, p=0.5,
                       kappa=0.6, lam=0.01)
    r = _hetero_oracle(oracle, g)
    base = oracle.sweep_baseline([1.0], 15.0, 30.0, g.u, 0.5, 0.6, 0.01)
    run_h = (r["status"] & 1) > 0
    run_b = (base["status"] & 1) > 0
    assert np.array_equal(run_h, run_b)
    assert np.nanmax(np.abs(r["xi"] - base["xi"])) < 1e-9


@pytest.mark.gpu
def test_hetero_gpu_bitwise_script_and_grid(engine, oracle):
    for g in (sbr.hetero_script_grid(), sbr.hetero_config4(24, 48, 8), sbr.hetero_config4(10, 30, 4),
              sbr.hetero_config4(8, 20, 2)):
        gg = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0)
        o = _hetero_oracle(oracle, g)
        for f in ("xi", "aw_max", "tol", "tau_in_unc", "tau_out_unc"):
            a, b = gg[f], o[f]
            same = (a == b) | (np.isnan(a) & np.isnan(b))
            assert same.all(), (g.name, f, int((~same).sum()))
        assert np.array_equal(gg["status"], o["status"]), g.name
        assert np.array_equal(gg["iters"], o["iters"]), g.name


@pytest.mark.gpu
def test_hetero_aw_branch_and_bound_equals_exhaustive(engine, oracle):
    """AW_max by branch and bound over the group CDFs (nondecreasing up to their ulp-sized
    drawdown in the saturated tail) == every knot evaluated (a different search, the same
    arithmetic), on a config-4 subgrid whose columns include such drawdowns."""
    g = sbr.hetero_config4(64, 96, 8)
    drawdown = 0
    for c in (0, 21, 42):
        _, G, _ = oracle.learn_hetero(g.betas[c], g.dist, g.t_end[c])
        drawdown += int((np.diff(G, axis=0) < 0).any())
    assert drawdown > 0  # the drawdown-tolerant bounds are exercised, not only the monotone case
    a = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False)
    b = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False,
                            exhaustive=True)
    for f in ("xi", "aw_max", "tol", "status", "iters"):
        assert np.array_equal(a[f], b[f], equal_nan=a[f].dtype.kind == "f"), f


@pytest.mark.gpu
def test_hetero_point_paths_bitwise(engine, oracle):
    """sbr_hetero_point_paths (the script point with its plotted paths: learning knots, the
    group CDFs, per-group buffers, AW_total and get_AW_hetero's per-group AW_OUT_k / AW_IN_k
    on the knots) == the oracle bit for bit."""
    g = sbr.hetero_script_grid()
    for u in (g.u[0], 0.9):
        a = engine.hetero_point_paths(g.betas[0], g.dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
        b = oracle.hetero_point_paths(g.betas[0], g.dist, g.eta[0], g.t_end[0], u, g.p, g.kappa, g.lam)
        assert a["status"] == b["status"], u
        for k in ("xi", "aw_max", "tol", "tau_in_unc", "tau_out_unc", "t", "G", "aw_total", "aw_out", "aw_in"):
            x, y = np.atleast_1d(a[k]), np.atleast_1d(b[k])
            assert x.shape == y.shape and np.array_equal(x, y, equal_nan=True), (u, k)
        if a["status"] & sbr.STATUS["SBR_RUN"]:
            assert np.max(a["aw_total"]) == a["aw_max"]


@pytest.mark.gpu
def test_learn_hetero_bitwise(engine, oracle):
    """sbr_learn_hetero (solve_SInetwork_hetero, run to t_end like the reference) == the
    oracle's knots and group CDFs, on the script column and two config-4 columns (one of
    which switches to Rosenbrock23)."""
    g = sbr.hetero_script_grid()
    c4 = sbr.hetero_config4(4, 4)
    cols = [(g.betas[0], g.dist, g.t_end[0])] + [(c4.betas[i], c4.dist, c4.t_end[i]) for i in (0, 3)]
    for betas, dist, t_end in cols:
        a = engine.learn_hetero(np.atleast_2d(betas), dist, t_end)
        t, G, st = oracle.learn_hetero(betas, dist, t_end)
        n = int(a["n_knots"][0])
        assert n == len(t), (betas, n, len(t))
        assert np.array_equal(a["t"][0, :n], t) and np.array_equal(a["G"][0, :n], G)
        assert int(a["status"][0]) & ~sbr.STATUS["SBR_STIFF_SWITCH"] == st["status"] & ~sbr.STATUS["SBR_STIFF_SWITCH"]


def test_hetero_point_paths_oracle_figure(oracle, golden):
    """The oracle's path output reproduces the script figure's AW_total maximum."""
    g = sbr.hetero_script_grid()
    r = oracle.hetero_point_paths(g.betas[0], g.dist, g.eta[0], g.t_end[0], g.u[0], g.p, g.kappa, g.lam)
    assert r["status"] & sbr.STATUS["SBR_RUN"]
    assert np.nanmax(r["aw_total"]) == r["aw_max"]
    assert r["G"].shape == (len(r["t"]), len(g.dist))
    # the per-group curves fold into AW_total in get_AW_hetero's order (:356-358: AW_cum .+=
    # dist[k] .* (AW_OUT_k .- AW_IN_k), k = 1..K), bit for bit
    cum = np.zeros(len(r["t"]))
    for k in range(len(g.dist)):
        cum = cum + g.dist[k] * (r["aw_out"][k] - r["aw_in"][k])
    assert np.array_equal(cum, r["aw_total"])
    # AW_OUT_k / AW_IN_k are group CDF values (0 where the shifted time is negative)
    assert (r["aw_out"] >= 0).all() and (r["aw_in"] >= 0).all() and (r["aw_in"] <= r["aw_out"] + 1e-12).all()


@pytest.mark.gpu
def test_hetero_reference_call_surface(engine, oracle):
    """scripts/2_heterogeneity.jl through the host mirror: ModelParametersHetero →
    solve_equilibrium_hetero (learning + equilibrium + AW paths) and get_AW_functions_hetero!
    (every curve from the engine), equal to the oracle."""
    g = sbr.hetero_script_grid()
    m = sbr.ModelParametersHetero.make(g.betas[0], g.dist, eta_bar=30.0, u=float(g.u[0]), p=g.p, kappa=g.kappa,
                                       lam=g.lam)
    r = sbr.solve_equilibrium_hetero(m, engine=engine)
    o = oracle.hetero_point_paths(g.betas[0], g.dist, m.economic.eta, m.learning.tspan[1], float(g.u[0]), g.p,
                                  g.kappa, g.lam)
    assert r.status == o["status"] and r.xi == o["xi"] and r.AW_max == o["aw_max"]
    assert np.array_equal(r.AW_total, o["aw_total"])
    aw = r.get_AW_functions_hetero()
    assert aw["AW_max"] == o["aw_max"] and np.array_equal(aw["AW_cum"].coefs, o["aw_total"])
    for k in range(len(g.dist)):
        assert np.array_equal(aw["AW_OUT_groups"][k].coefs, o["aw_out"][k]), k
        assert np.array_equal(aw["AW_IN_groups"][k].coefs, o["aw_in"][k]), k
        assert np.array_equal(aw["AW_groups"][k].coefs, o["aw_out"][k] - o["aw_in"][k]), k


@pytest.mark.gpu
def test_hetero_pipelined_batches_equal_single_sweeps(engine):
    """sbr_sweep_hetero_batch_dev (learning of batch k+1 on a second stream into the other
    workspace while batch k's equilibrium runs) returns for every batch exactly what
    sbr_sweep_hetero returns for that grid."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    full = sbr.hetero_config4(96, 40, 8)
    subs = [full.subset(np.arange(k, 96, 3)) for k in range(3)]  # three 32-column grids
    nbat, nc, nu, K = len(subs), 32, len(full.u), full.K
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {f: torch.empty(nbat, nc * nu, dtype=torch.float64, device=dev) for f in ("xi", "aw_max", "tol")}
    out["status"] = torch.empty(nbat, nc * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nbat, nc * nu, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    engine.sweep_hetero_batch_dev(K, t(np.stack([g.betas for g in subs])), t(full.dist),
                                  t(np.stack([g.eta for g in subs])), t(np.stack([g.t_end for g in subs])),
                                  t(full.u), full.p, full.kappa, full.lam, full.x0, out, stream=stream)
    torch.cuda.synchronize(dev)
    for k, g in enumerate(subs):
        ref = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False)
        for f in ("xi", "aw_max", "tol"):
            a = out[f][k].cpu().numpy().reshape(nc, nu)
            assert np.array_equal(a, ref[f].reshape(nc, nu), equal_nan=True), (k, f)
        assert np.array_equal(out["status"][k].cpu().numpy().view(np.uint32).reshape(nc, nu),
                              ref["status"].reshape(nc, nu)), k
        assert np.array_equal(out["iters"][k].cpu().numpy().reshape(nc, nu), ref["iters"].reshape(nc, nu)), k


@pytest.mark.gpu
def test_hetero_batch_ordered_on_torch_default_stream(engine):
    """A batch enqueued on torch's default stream (handle 0, HIP's null stream) is complete
    for torch work enqueued on that stream afterwards, with no host synchronisation in
    between (bench.py copies the last batch's status this way)."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    g = sbr.hetero_config4(64, 48, 8)
    nbat, nc, nu, K = 2, 64, len(g.u), g.K
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {f: torch.zeros(nbat, nc * nu, dtype=torch.float64, device=dev) for f in ("xi", "aw_max", "tol")}
    out["status"] = torch.zeros(nbat, nc * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.zeros(nbat, nc * nu, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    assert stream == 0
    rep = lambda a: t(np.stack([a] * nbat))
    engine.sweep_hetero_batch_dev(K, rep(g.betas), t(g.dist), rep(g.eta), rep(g.t_end), t(g.u), g.p, g.kappa,
                                  g.lam, g.x0, out, stream=stream)
    st = out["status"][nbat - 1].clone()  # enqueued behind the batch on the same stream
    aw = out["aw_max"][nbat - 1].clone()
    torch.cuda.synchronize(dev)
    ref = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False)
    assert np.array_equal(st.cpu().numpy().view(np.uint32), ref["status"].ravel())
    assert np.array_equal(aw.cpu().numpy(), ref["aw_max"].ravel(), equal_nan=True)


@pytest.mark.gpu
def test_hetero_config4_full_properties_and_strided_columns(engine, oracle):
    """BASELINE config 4 at its stated size (K = 8, 1024 × 1024 = 1,048,576 equilibria) on
    the GPU: every learning column switches to Rosenbrock23 (AutoSwitch, handled); size-
    independent properties over the whole grid; 128 strided columns (every 8th, all 1024 u:
    131,072 equilibria, 12.5 % of the grid) bit for bit against the oracle's sweep_hetero."""
    g = sbr.hetero_config4(1024, 1024, 8)
    r = engine.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False)
    st = r["status"]
    run = (st & sbr.STATUS["SBR_RUN"]) > 0
    # every column's AutoSwitch moves to Rosenbrock23 at least once (the stiff branch runs)
    assert ((st & sbr.STATUS["SBR_STIFF_SWITCH"]) > 0).all()
    assert not (st & (sbr.STATUS["SBR_ODE_FAILED"] | sbr.STATUS["SBR_ODE_MAXITERS"] | sbr.STATUS["SBR_KNOT_OVERFLOW"]
                      | sbr.STATUS["SBR_ENGINE_TRUNC"])).any()
    # points whose bisection probes ξ + Δt past the last knot (t_end) are where the reference's
    # LinearInterpolation raises BoundsError (no try/catch in the reference): the oracle flags the
    # same ~4 % of this grid (every 37th u, all 1024 columns: 1118 of 28672), so they are reported,
    # not failures; nothing else rides on them
    oob = (st & sbr.STATUS["SBR_OOB"]) > 0
    assert oob.mean() < 0.1
    assert (st[oob] == sbr.STATUS["SBR_OOB"] | sbr.STATUS["SBR_STIFF_SWITCH"]).all()
    assert np.isnan(r["xi"][oob]).all() and np.isnan(r["aw_max"][oob]).all()
    # SolvedModel conventions: ξ / AW_max finite exactly on run points, tol Inf off them
    assert np.isfinite(r["xi"][run]).all() and np.isnan(r["xi"][~run]).all()
    assert np.isfinite(r["aw_max"][run]).all() and np.isnan(r["aw_max"][~run]).all()
    assert (r["tol"][run] <= 1e-12).all()
    no_trivial = (st & sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"]) > 0
    assert (r["tol"][no_trivial] == 0.0).all() and np.isinf(r["tol"][~run & ~no_trivial]).all()
    # AW(ξ*) = κ within the bisection tolerance, so the path maximum is at least κ
    assert (r["aw_max"][run] >= g.kappa - 1e-12).all()
    assert 0.5 < run.mean() < 1.0
    # 128 strided columns (every 8th), every u, bit for bit
    sub = g.subset(np.arange(0, 1024, 8))
    o = oracle.sweep_hetero(sub.betas, sub.dist, sub.eta, sub.t_end, sub.u, sub.p, sub.kappa, sub.lam, sub.x0,
                            nthreads=16)
    for f in ("xi", "aw_max", "tol", "status", "iters"):
        a, b = r[f][::8], o[f]
        same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
        assert same.all(), (f, int((~same).sum()))
    # the learning of a strided column: knots bit for bit, Rosenbrock23 steps taken
    t_o, G_o, info = oracle.learn_hetero(g.betas[512], g.dist, g.t_end[512])
    assert info["nswitch"] > 0 and info["nstiff"] > 0
