"""GPU parity: the gfx950 kernels, called through libsbr's C ABI, against the
CPU oracle on the same inputs — bit for bit — and against the reference's
golden figures at full size."""
import numpy as np
import pytest

import sbr

pytestmark = pytest.mark.gpu

FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")


def assert_bitwise(a, b, name):
    a = np.asarray(a)
    b = np.asarray(b)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    if not same.all():
        idx = np.argwhere(~same)[:5]
        raise AssertionError(f"{name}: {int((~same).sum())} mismatches, e.g. {[(tuple(i), a[tuple(i)], b[tuple(i)]) for i in idx]}")


def test_detmath_host_device_bitwise(engine, oracle):
    rng = np.random.default_rng(0)
    # sbr_exp's device fast path (x = 0 or 2^-400 <= |x| <= 708) and the full branch-free
    # form around its edges, the hazard's λτ̄ range, and every k's reduction boundary
    edges = np.array([708.0, -708.0, np.nextafter(708.0, 1e3), np.nextafter(-708.0, -1e3), 2.0 ** -400,
                      -(2.0 ** -400), np.nextafter(2.0 ** -400, 0.0), 5e-324, -5e-324, 709.78, -745.1, np.inf,
                      -np.inf, np.nan, -0.0])
    ks = np.arange(-1030, 1030) * np.log(2.0)
    x = np.concatenate([rng.uniform(-745, 709, 20000), np.exp(rng.uniform(-700, 700, 20000)),
                        rng.uniform(1e-300, 1e-290, 100), [0.0, 1.0, 2.0, 0.5], edges, ks,
                        np.nextafter(ks, np.inf), np.nextafter(ks, -np.inf), ks + np.log(2.0) / 2,
                        rng.uniform(0.0, 8.0, 20000)])
    y = rng.uniform(-1.0, 1.0, len(x))
    xe = x.copy()
    e_d, _, _ = engine.selftest_detmath(xe, y)
    e_h, _, _ = oracle.detmath(xe, y)
    assert_bitwise(e_d, e_h, "exp")
    xp = np.abs(x) + 1e-300
    _, l_d, p_d = engine.selftest_detmath(xp, y)
    _, l_h, p_h = oracle.detmath(xp, y)
    assert_bitwise(l_d, l_h, "log")
    assert_bitwise(p_d, p_h, "pow")


@pytest.mark.parametrize("stop", [False, True])
def test_learning_knots_bitwise(engine, oracle, stop):
    """Every knot (t, G) of the device integrator equals the oracle's; the
    truncated mode (stop after the last knot the equilibrium can read) is a
    prefix of the full solve."""
    grid = sbr.fig5_grid(500)
    betas = np.concatenate([grid.beta[::25], [0.5, 1.0, 2.0, 3.0, 61.654026637430945]])
    res = engine.learn_baseline(betas, 15.0, 30.0, stop_after_eta=stop)
    for b, (t, G, st) in zip(betas, res):
        to, Go, sto = oracle.learn_logistic(float(b), 30.0)
        if stop:
            assert len(t) <= len(to) and t[-1] > 15.0
        else:
            assert len(t) == len(to)
        assert_bitwise(t, to[: len(t)], f"t β={b}")
        assert_bitwise(G, Go[: len(t)], f"G β={b}")


@pytest.mark.parametrize("tol", [1e-10, 1e-6])
def test_learning_tol_bitwise(engine, oracle, tol):
    """solve_learning(lp; tol) (learning.jl:109, reltol = abstol = tol in solve_SIhomogeneous
    :41-51): the drop-ins pass the keyword through (julia/SBRDropIn.jl), and the device knots at a
    looser tolerance equal the oracle's, knot for knot."""
    for b in (0.5, 1.0, 3.0, 61.654026637430945):
        lr = sbr.solve_learning(sbr.LearningParameters(b, (0.0, 30.0), 1e-4), engine, tol=tol)
        to, Go, _ = oracle.learn_logistic(float(b), 30.0, rtol=tol, atol=tol)
        assert len(lr.grid) == len(to)
        assert_bitwise(lr.grid, to, f"t β={b}")
        assert_bitwise(lr.learning_cdf.coefs, Go, f"G β={b}")


def _oracle_sweep(oracle, grid):
    return oracle.sweep_baseline(grid.beta, grid.eta, grid.t_end, grid.u, grid.p, grid.kappa, grid.lam, grid.x0)


def test_fig5_500_sweep_bitwise(engine, oracle, golden):
    """All 250,000 points of the Fig 5 grid: every output field and status bit
    identical to the oracle; run mask identical to the committed heatmap."""
    grid = sbr.fig5_grid(500)
    g = engine.sweep_baseline(grid)
    o = _oracle_sweep(oracle, grid)
    for f in FIELDS:
        assert_bitwise(g[f], o[f], f)
    assert np.array_equal(g["status"], o["status"])
    assert np.array_equal(g["iters"], o["iters"])
    run = (g["status"] & sbr.STATUS["SBR_RUN"]) > 0
    assert run.sum() == golden("fig5_prefix.json")["n500"]["total"]


def test_sweep_into_caller_arrays(engine, oracle):
    """sweep_baseline(out=...) fills the caller's arrays in place (the config-2 bench path),
    call after call, with the oracle's bits; wrong dtypes or sizes are refused before the call."""
    grid = sbr.fig5_grid(96)
    n = grid.n_points
    host = {f: np.full(n, -1.0) for f in FIELDS}
    host["status"] = np.zeros(n, np.uint32)
    host["iters"] = np.zeros(n, np.int32)
    o = _oracle_sweep(oracle, grid)
    for _ in range(2):
        r = engine.sweep_baseline(grid, out=host)
        assert np.shares_memory(r["xi"], host["xi"])
        for f in FIELDS:
            assert_bitwise(host[f].reshape(o[f].shape), o[f], f)
        assert np.array_equal(host["status"].reshape(o["status"].shape), o["status"])
        host["xi"][:] = 0.0
    bad = dict(host, status=np.zeros(n, np.int64))
    with pytest.raises(sbr.ArgumentError):
        engine.sweep_baseline(grid, out=bad)
    with pytest.raises(sbr.ArgumentError):
        engine.sweep_baseline(grid, out=dict(host, xi=np.zeros(n - 1)))


def test_fig4_sweep_bitwise_and_boundary(engine, oracle, golden):
    grid = sbr.fig4_grid(5000)
    g = engine.sweep_baseline(grid, early_exit=5)
    o = oracle.apply_early_exit(_oracle_sweep(oracle, grid), 5)
    for f in FIELDS:
        assert_bitwise(g[f], o[f], f)
    assert np.array_equal(g["status"], o["status"])
    run = (g["status"][0] & sbr.STATUS["SBR_RUN"]) > 0
    n = golden("fig4_u_sweep.json")["n_run_prefix"]
    assert run[:n].all() and not run[n:].any()


@pytest.mark.parametrize("case", ["main", "fast", "low_u"])
def test_point_paths_bitwise(engine, oracle, golden, case):
    """Single-point mode (τ̄, HR(τ̄), AW_cum(τ̄)) equals the oracle and hits Fig 3."""
    P = golden("fig3_equilibria.json")[case]["params"]
    r = engine.solve_point_paths(P["beta"], P["eta"], P["t_end"], P["u"], P["p"], P["kappa"], P["lam"])
    t, G, _ = oracle.learn_logistic(P["beta"], P["t_end"])
    o = oracle.equilibrium(t, G, P["beta"], P["eta"], P["t_end"], P["u"], P["p"], P["kappa"], P["lam"], paths=True)
    assert r["status"] == o["status"]
    for f in FIELDS:
        assert_bitwise(r[f], o[f], f)
    assert_bitwise(r["tau"], o["hr_tau"], "tau")
    assert_bitwise(r["hr"], o["hr"], "hr")
    assert_bitwise(r["aw_cum"], o["aw"], "aw_cum")
    gx = golden("fig3_equilibria.json")[case]
    assert abs(r["xi"] - gx["xi"]) <= 1.5 * gx["xi_precision"] + 2e-5


def test_reference_call_surface(engine):
    """solve_learning → solve_equilibrium_baseline → get_AW_functions on the GPU."""
    m = sbr.ModelParameters.make(beta=1.0, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
    lr = sbr.solve_learning(m.learning, engine)
    res = sbr.solve_equilibrium_baseline(lr, m.economic, engine)
    assert res.bankrun and res.converged
    aw = sbr.get_AW_functions(res)
    assert abs(aw["AW_max"] - 0.6182312) < 1e-6
    assert abs(aw["AW_cum"](0.0) - 2e-4) < 1e-12  # AW_cum(0) = 2 x0 (solver.jl:523-524)
    assert abs(res.tau_IN - 2.8879) < 2e-4


def test_config3_2048_properties_and_columns(engine, oracle):
    """Benchmark config 3 (2048², 4.19M points): spot columns bitwise against
    the oracle plus size-independent properties on the whole grid."""
    grid = sbr.fig5_grid(2048)
    g = engine.sweep_baseline(grid)
    st = g["status"]
    run = (st & sbr.STATUS["SBR_RUN"]) > 0
    bad = sbr.STATUS["SBR_ENGINE_TRUNC"] | sbr.STATUS["SBR_KNOT_OVERFLOW"] | sbr.STATUS["SBR_OOB"]
    assert not (st & bad).any()
    # outcome classes are exclusive and exhaustive
    cls = (sbr.STATUS["SBR_RUN"] | sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"] | sbr.STATUS["SBR_NO_RUN_COLLAPSE"]
           | sbr.STATUS["SBR_NO_RUN_MAXITER"] | sbr.STATUS["SBR_FALSE_EQ"])
    assert ((st & cls) != 0).all()
    # run ⇔ finite ξ; aw_max ≥ κ − tol on runs (AW reaches κ at ξ); ξ within the buffers
    assert np.array_equal(run, np.isfinite(g["xi"]))
    assert (g["aw_max"][run] >= 0.6 - 1e-12).all()
    assert ((g["xi"][run] >= g["tau_in_unc"][run]) & (g["xi"][run] <= g["tau_out_unc"][run])).all()
    assert (g["tol"][run] <= 10 * np.spacing(0.6)).all()
    # run cells form a u-prefix in every β column (what the Fig 5 masks show)
    for c in range(run.shape[0]):
        k = np.argmin(run[c]) if not run[c].all() else run.shape[1]
        assert run[c, :k].all() and not run[c, k:].any()
    cols = np.random.default_rng(0).choice(2048, 12, replace=False)
    sub = grid.subset(np.sort(cols))
    o = _oracle_sweep(oracle, sub)
    for f in FIELDS:
        assert_bitwise(g[f][np.sort(cols)], o[f], f)
    assert np.array_equal(st[np.sort(cols)], o["status"])


def test_fig5_5000_run_mask(engine, golden):
    """Paper resolution (5000², 25M points, scripts/1_baseline.jl:208): the run
    mask of comp_stat_cross_heatmap_AW_large.pdf column by column (8,736,564 cells)."""
    grid = sbr.fig5_grid(5000)
    pref = np.array(golden("fig5_prefix.json")["n5000"]["prefix"])
    g = engine.sweep_baseline(grid, early_exit=5, with_iters=False)
    run = (g["status"] & sbr.STATUS["SBR_RUN"]) > 0
    got = np.array([np.argmin(r) if not r.all() else len(r) for r in run])
    assert np.array_equal(got, pref), f"{int((got != pref).sum())} columns differ"
    assert run.sum() == 8736564


@pytest.mark.parametrize("case", ["single_point", "ragged_extremes", "eta_past_tend", "short_eta_per_column"])
def test_edge_grids_bitwise(engine, oracle, case):
    """Edge shapes and parameter extremes, every field, status bit and bisection count
    equal to the oracle: a 1 × 1 grid; 6 × 65 (partial waves and tiles) with β from 1e-3 to
    3e4 and u from 0 to 1.5 (no-run, run and u > every HR value); η beyond tspan on one
    column (the reference's BoundsError); per-column η and t_end."""
    if case == "single_point":
        g = sbr.BaselineGrid([1.0], [0.05], 15.0, 30.0)
    elif case == "ragged_extremes":
        g = sbr.BaselineGrid([1e-3, 0.2, 7.3, 250.0, 1e4, 3e4], sbr.julia_range("0.0", "1.5", 65), 15.0, 30.0)
    elif case == "eta_past_tend":
        g = sbr.BaselineGrid([0.5, 2.0, 2.0], sbr.julia_range("0.001", "1", 97), np.array([40.0, 15.0, 30.0]),
                             np.array([30.0, 30.0, 30.0]))
    else:
        g = sbr.BaselineGrid([0.7, 1.3, 4.0, 12.0, 40.0], sbr.julia_range("0.001", "1", 130),
                             np.array([0.5, 3.0, 9.0, 15.0, 20.0]), np.array([1.0, 10.0, 18.0, 30.0, 60.0]))
    a = engine.sweep_baseline(g)
    o = _oracle_sweep(oracle, g)
    for f in FIELDS:
        assert_bitwise(a[f], o[f], f"{case} {f}")
    assert np.array_equal(a["status"], o["status"]), case
    assert np.array_equal(a["iters"], o["iters"]), case
    if case == "eta_past_tend":
        assert (a["status"][0] & sbr.STATUS["SBR_OOB"]).all()


def test_blocked_scan_and_pruned_aw_equal_exhaustive(engine):
    """Block-summary crossing scan + branch-and-bound AW_max give exactly the
    exhaustive per-knot results (a different search, the same arithmetic)."""
    for grid in (sbr.fig5_grid(512), sbr.fig4_grid(5000), sbr.BaselineGrid([0.5, 1.0, 3.0, 61.654026637430945], sbr.julia_range("0.0", "2.0", 777), 15.0, 30.0, p=1.0)):
        a = engine.sweep_baseline(grid)
        b = engine.sweep_baseline(grid, exhaustive=True)
        for f in FIELDS:
            assert_bitwise(a[f], b[f], f)
        assert np.array_equal(a["status"], b["status"])
        assert np.array_equal(a["iters"], b["iters"])


def test_device_info(engine):
    info = engine.device_info()
    assert info["cu_count"] == 256
    assert info["lds_knot_capacity"] >= 3400  # every config-3 column staged in LDS


@pytest.mark.parametrize("ncol,group", [(384, None), (1200, None), (1536, None), (384, 3), (1200, 2)])
def test_pipelined_batches_equal_single_sweeps(engine, ncol, group):
    """sbr_sweep_baseline_batch_dev returns for every batch exactly what a single sweep of that
    grid returns.  By default the 11 grids are learned in one launch (≤ one wave per SIMD) and
    solved by equilibrium launches of ⌈4096 / n_β⌉ grids (384 columns: 11 grids in one launch;
    1200: three launches of 4, 4, 3).  The learning launch deals every grid's first wave first
    where grids are whole waves (384: 6 waves per grid, 1536: 24) and stages its rows through LDS
    from 256 waves on (1536: 264 waves, the wide launch of the config-3 bench).  With a workspace budget of `group` grids per learning
    launch (sbr_set_batch_workspace) the batch runs in groups — 384: four groups of 3, 3, 3, 2;
    1200: six of 2, ..., 1 — learned into two alternating workspaces, each group beside the
    previous group's equilibria, so each workspace is reused behind its readers."""
    torch = pytest.importorskip("torch")
    if group is not None:
        # two workspaces of `group` grids: n_β × (4 × cap × 8 + 24) bytes per grid
        engine.set_batch_workspace(2 * group * ncol * (4 * 65536 * 8 + 24) + 4096)
    dev = torch.device("cuda", 0)
    base = sbr.fig5_grid(ncol, n_u=384)
    betas = np.stack([base.beta, base.beta[::-1], base.beta * 0.5, base.beta])
    etas = np.stack([np.full(ncol, 15.0), np.full(ncol, 10.0), np.full(ncol, 15.0), np.full(ncol, 7.5)])
    etas[1, :7] = 40.0  # η past tspan: the hazard stage's BoundsError (fused into learning in the batch)
    etas[2, 7:9] = 30.0  # η == t_end: the last knot is η itself
    tends = np.stack([np.full(ncol, 30.0), np.full(ncol, 30.0), np.full(ncol, 20.0), np.full(ncol, 30.0)])
    # 11 grids; the extra grids vary β so no two are alike
    extra = np.arange(7)[:, None]
    betas = np.concatenate([betas, base.beta[None, :] * (1.0 + 0.05 * (extra + 1))])
    etas = np.concatenate([etas, np.full((7, ncol), 15.0) - extra])
    tends = np.concatenate([tends, np.full((7, ncol), 30.0)])
    nbat, nb, nu = betas.shape[0], betas.shape[1], len(base.u)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {f: torch.empty(nbat, nb * nu, dtype=torch.float64, device=dev) for f in FIELDS}
    out["status"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    engine.sweep_baseline_batch_dev(t(betas), t(etas), t(tends), t(base.u), base.p, base.kappa, base.lam, base.x0,
                                    out, stream=stream)
    # enqueued behind the call on torch's default stream, no host synchronisation between:
    # must see every batch complete (whichever equilibrium stream ran it)
    snap = {f: out[f].clone() for f in ("aw_max", "status")}
    # grid k shipped from a side stream ordered only by sbr_batch_wait (bench.py's gathers)
    side = torch.cuda.Stream(dev)
    early = []
    for k in range(nbat):
        engine.batch_wait(side.cuda_stream, k)
        with torch.cuda.stream(side):
            early.append(out["aw_max"][k].clone())
    with pytest.raises(sbr.ArgumentError):
        engine.batch_wait(side.cuda_stream, nbat)
    torch.cuda.synchronize(dev)
    for k in range(nbat):
        assert torch.equal(early[k].view(torch.int64), out["aw_max"][k].view(torch.int64)), k
    for f in snap:
        assert torch.equal(snap[f].view(torch.int64) if f == "aw_max" else snap[f],
                           out[f].view(torch.int64) if f == "aw_max" else out[f]), f
    for k in range(nbat):
        g = sbr.BaselineGrid(betas[k], base.u, etas[k], tends[k], x0=base.x0, p=base.p, kappa=base.kappa,
                             lam=base.lam)
        ref = engine.sweep_baseline(g)
        for f in FIELDS:
            assert_bitwise(out[f][k].cpu().numpy().reshape(nb, nu), ref[f], f"batch {k} {f}")
        st = out["status"][k].cpu().numpy().view(np.uint32).reshape(nb, nu)
        assert np.array_equal(st, ref["status"])
        assert np.array_equal(out["iters"][k].cpu().numpy().reshape(nb, nu), ref["iters"])
    engine.set_batch_workspace(0)


def test_batch_workspace_allocation_falls_back(engine):
    """A batch whose planned workspace does not fit the device (budget lifted, a 20M-knot
    capacity: 41 GB per 64-column grid, 8 grids planned into one 328 GB workspace) halves its
    learning group until the allocation succeeds — here two workspaces of two
    grids — and still returns every grid exactly as single sweeps do.  sbr_batch_reserve takes
    the same path.  Own context: the 164 GB are released at the end."""
    torch = pytest.importorskip("torch")
    dev = torch.device("cuda", 0)
    cap = 20_000_000
    base = sbr.fig5_grid(64, n_u=64)
    nbat = 8
    betas = np.stack([base.beta * (1.0 + 0.03 * k) for k in range(nbat)])
    eta = np.full((nbat, 64), 15.0)
    tend = np.full((nbat, 64), 30.0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    out = {f: torch.empty(nbat, 64 * 64, dtype=torch.float64, device=dev) for f in FIELDS}
    out["status"] = torch.empty(nbat, 64 * 64, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nbat, 64 * 64, dtype=torch.int32, device=dev)
    eng = sbr.Engine(0)
    try:
        eng.set_batch_workspace(1 << 50)
        eng.batch_reserve(nbat, 64, knot_capacity=cap)
        eng.sweep_baseline_batch_dev(t(betas), t(eta), t(tend), t(base.u), base.p, base.kappa, base.lam, base.x0,
                                     out, knot_capacity=cap)
        torch.cuda.synchronize(dev)
    finally:
        eng.close()
    for k in (0, 3, nbat - 1):
        g = sbr.BaselineGrid(betas[k], base.u, eta[k], tend[k], x0=base.x0, p=base.p, kappa=base.kappa,
                             lam=base.lam)
        ref = engine.sweep_baseline(g)
        for f in FIELDS:
            assert_bitwise(out[f][k].cpu().numpy().reshape(64, 64), ref[f], f"batch {k} {f}")
        assert np.array_equal(out["status"][k].cpu().numpy().view(np.uint32).reshape(64, 64), ref["status"])


@pytest.mark.parametrize("n_u", [50, 9000])
def test_readiness_schedule_equals_chunked(engine, n_u):
    """The per-column readiness schedule (SBR_FLAG_READY_SWEEP: the learning kernel publishes
    each column the moment its lane solves it; equilibrium workgroups on other CUs take
    (column, u-tile) items in publication order, tile 0 running the column's hazard) gives
    exactly the default three-chunk schedule's results — incl. BoundsError columns (η past
    tspan), η == t_end, and one u-tile per column (n_u = 50) or three (n_u = 9000 > 2 × 4096:
    tiles 1 and 2 wait on the tile-0 workgroup's hazard flag).  The schedule is asserted taken."""
    base = sbr.fig5_grid(384, n_u=n_u)
    eta = np.full(384, 15.0)
    tend = np.full(384, 30.0)
    eta[:5] = 40.0   # η past tspan: the hazard's BoundsError
    eta[100:103] = 30.0  # η == t_end: η is the last knot
    tend[200:210] = 20.0
    g = sbr.BaselineGrid(base.beta, base.u, eta, tend)
    a = engine.sweep_baseline(g, flags=sbr._lib.SBR_FLAG_READY_SWEEP)
    assert engine.last_schedule() == 1  # the MI355X (256 CUs) runs the readiness schedule
    b = engine.sweep_baseline(g)
    assert engine.last_schedule() == 0
    for f in FIELDS:
        assert_bitwise(a[f], b[f], f)
    assert np.array_equal(a["status"], b["status"])
    assert np.array_equal(a["iters"], b["iters"])
    assert (a["status"][:5] & sbr.STATUS["SBR_OOB"]).all()
    # and repeatedly (the publication queue is reset per call)
    c = engine.sweep_baseline(g, flags=sbr._lib.SBR_FLAG_READY_SWEEP)
    assert np.array_equal(c["status"], a["status"]) and np.array_equal(c["aw_max"], a["aw_max"], equal_nan=True)
