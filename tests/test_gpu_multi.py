"""Multi-GPU fan-out inside libsbr (sbr_init_multi, include/sbr.h; SURVEY.md §8(b)
threading contract, §8(e) partitioning): an n-device context deals the parameter
columns cyclically over its GPUs, one host thread per GPU, and returns each rank's result
block over its own link (pinned landing buffer, then host threads into the caller's arrays;
SBR_FLAG_RCCL_GATHER: an RCCL gather to device 0 instead).  On the one-GPU test box n = 1
(the rank threads, both transports and the strided scatter all run); the multi-rank column
interleaving of the Python layer is covered by the world-2/3 gloo tests of
tests/test_distributed.py.  Every result must equal the single-device context's bit
for bit, and the engine-backed sbr.distributed sweeps (compute=None) must run."""
import ctypes

import numpy as np
import pytest

import sbr
from sbr import _lib

pytestmark = pytest.mark.gpu

FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")


def _n_gpus():
    import torch

    return torch.cuda.device_count()


def assert_same(a, b, name):
    a, b = np.asarray(a), np.asarray(b)
    same = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else (a == b)
    assert same.all(), f"{name}: {int((~same).sum())} mismatches"


@pytest.fixture(scope="module")
def multi():
    return sbr.Engine(n_gpus=_n_gpus())


def test_multi_context_ccall_style(engine):
    """The C ABI exactly as a Julia `ccall` would bind it: sbr_init_multi, a host-pointer
    sweep (Fig 5 columns), sbr_multi_size / sbr_multi_child, the device-pointer guard."""
    L = _lib.load()
    n = _n_gpus()
    ctx = ctypes.c_void_p()
    assert L.sbr_init_multi(n, None, ctypes.byref(ctx)) == 0
    try:
        assert L.sbr_multi_size(ctx) == n
        assert L.sbr_multi_child(ctx, 0) and not L.sbr_multi_child(ctx, n)
        g = sbr.fig5_grid(500)
        sub = g.subset(np.arange(0, 500, 7))
        nb, nu = len(sub.beta), len(sub.u)
        out = {k: np.empty(nb * nu) for k in FIELDS}
        out["status"] = np.empty(nb * nu, np.uint32)
        out["iters"] = np.empty(nb * nu, np.int32)
        soa = _lib.ResultSoA(*[out[k].ctypes.data_as(ctypes.c_void_p) for k in (*FIELDS, "status", "iters")])
        opts = _lib.default_opts(early_exit_nan_run=0)
        P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        rc = L.sbr_sweep_baseline(ctx, P(sub.beta), P(sub.eta), P(sub.t_end), sub.x0, P(sub.u), nb, nu, sub.p,
                                  sub.kappa, sub.lam, ctypes.byref(opts), ctypes.byref(soa))
        assert rc == 0, L.sbr_last_error(ctx)
        ref = engine.sweep_baseline(sub)
        for k in (*FIELDS, "status", "iters"):
            assert_same(out[k].reshape(nb, nu), ref[k], k)
        # device pointers belong to one GPU: an n-device context refuses them
        rc = L.sbr_sweep_baseline_dev(ctx, None, None, None, None, 1e-4, None, 1, 1, 0.5, 0.6, 0.01,
                                      ctypes.byref(opts), ctypes.byref(soa))
        assert rc == _lib.SBR_EARG and b"single-device" in L.sbr_last_error(ctx)
    finally:
        L.sbr_free(ctx)


@pytest.mark.parametrize("flags", [0, _lib.SBR_FLAG_RCCL_GATHER], ids=["direct", "rccl_gather"])
def test_multi_baseline_fig5_and_early_exit(engine, multi, flags):
    """Both result transports of an n-device context (each rank's own D2H; the RCCL gather to
    device 0 then one scatter) give the single-device arrays."""
    g = sbr.fig5_grid(500)
    for ee in (0, 5):
        a = multi.sweep_baseline(g, early_exit=ee, flags=flags)
        b = engine.sweep_baseline(g, early_exit=ee)
        for k in (*FIELDS, "status", "iters"):
            assert_same(a[k], b[k], f"{k} (early_exit={ee})")


def test_multi_phases_recorded(multi):
    """sbr_host_phases on an n-device context: the fan-out's phases of the last sweep."""
    g = sbr.fig5_grid(500).subset(np.arange(0, 500, 5))
    multi.sweep_baseline(g)
    ph = multi.host_phases()
    assert set(ph) == {"slowest_rank_sweep", "slowest_rank_d2h_pinned", "host_copy_or_gather", "unused", "call"}
    assert ph["slowest_rank_sweep"] > 0 and ph["slowest_rank_d2h_pinned"] > 0 and ph["host_copy_or_gather"] > 0
    assert ph["call"] >= ph["slowest_rank_sweep"]


def test_multi_hetero_interest_social_bitwise(engine, multi):
    h = sbr.hetero_config4(1024, 64).subset(np.arange(0, 1024, 97))
    a = multi.sweep_hetero(h.betas, h.dist, h.eta, h.t_end, h.u, h.p, h.kappa, h.lam, h.x0)
    b = engine.sweep_hetero(h.betas, h.dist, h.eta, h.t_end, h.u, h.p, h.kappa, h.lam, h.x0)
    for k in ("xi", "aw_max", "tol", "status", "iters", "tau_in_unc", "tau_out_unc"):
        assert_same(a[k], b[k], f"hetero {k}")
    beta = 1.0 / sbr.julia_range("0.0001", "1", 60)
    u = sbr.julia_range("0.001", "1", 40)
    a = multi.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
    b = engine.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
    for k in (*FIELDS, "status", "iters", "rk_steps"):
        assert_same(a[k], b[k], f"interest {k}")
    eta = 30.0 / 0.9
    bs = 1.0 / sbr.julia_range("0.01", "2", 512)[[0, 200, 511]]
    us = sbr.julia_range("0.001", "1", 512)[[10, 300]]
    a = multi.sweep_social(bs, eta, us, 0.99, 0.25, 0.25, max_iter=3)
    b = engine.sweep_social(bs, eta, us, 0.99, 0.25, 0.25, max_iter=3)
    for k in (*FIELDS, "status", "iters", "fp_iters", "rk_steps"):
        assert_same(a[k], b[k], f"social {k}")


def test_engine_backed_sharded_sweeps_world1(engine):
    """sbr.distributed's sweeps with compute=None run libsbr (default_engine) at world 1."""
    from sbr import distributed as D

    g = sbr.fig5_grid(500).subset(np.arange(0, 500, 25))
    a = D.sweep_baseline_sharded(g)
    b = engine.sweep_baseline(g)
    for k in (*FIELDS, "status"):
        assert_same(a[k], b[k], f"sharded baseline {k}")
    h = sbr.hetero_config4(1024, 32).subset(np.arange(0, 1024, 211))
    a = D.sweep_hetero_sharded(h)
    b = engine.sweep_hetero(h.betas, h.dist, h.eta, h.t_end, h.u, h.p, h.kappa, h.lam, h.x0)
    for k in ("xi", "aw_max", "status"):
        assert_same(a[k], b[k], f"sharded hetero {k}")
    beta = 1.0 / sbr.julia_range("0.0001", "1", 20)
    u = sbr.julia_range("0.001", "1", 16)
    a = D.sweep_interest_sharded(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
    b = engine.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
    assert_same(a["aw_max"], b["aw_max"], "sharded interest aw_max")
    a = D.sweep_social_sharded([0.9, 2.0], 30.0 / 0.9, [0.5, 0.9], 0.99, 0.25, 0.25, max_iter=2)
    b = engine.sweep_social([0.9, 2.0], 30.0 / 0.9, [0.5, 0.9], 0.99, 0.25, 0.25, max_iter=2)
    assert_same(a["aw_max"], b["aw_max"], "sharded social aw_max")


def test_fastpow_host_device_bitwise(engine, oracle):
    """FastPower.fastpower (the PI controller's Float32 power) on the device == the oracle,
    over the controller's arguments (EEst^(7/50), qold^(2/25)) and edge values."""
    rng = np.random.default_rng(1)
    x = np.concatenate([np.exp(rng.uniform(-700, 5, 40000)), rng.uniform(1e-4, 2.0, 20000),
                        [1e-4, 1.0, 0.5, 1.5, 1e-45, 1e-40, 3e38, np.inf]])
    for y in (0.14, 0.08):
        assert_same(engine.selftest_fastpow(x, np.full(len(x), y)), oracle.fastpow(x, y), f"fastpow y={y}")


@pytest.mark.parametrize("n", [2, 3, 8])
def test_multi_rank_rehearsal_on_shared_device(engine, monkeypatch, n):
    """The n-rank fan-out on the one-GPU box (SBR_MULTI_SHARED_DEVICES=1: n ranks on device 0):
    n host threads, n child contexts and streams, per-rank pinned landing buffers, the cyclic
    deal with strided D2H and the all-or-nothing host scatter — the code an n-GPU node runs
    with the direct transport — bitwise equal to the single-device context for the baseline
    (with and without the 5-NaN early exit), hetero, interest and social sweeps.  The RCCL
    gather needs distinct devices and is refused here, leaving the caller's arrays untouched."""
    monkeypatch.setenv("SBR_MULTI_SHARED_DEVICES", "1")
    m = sbr.Engine(n_gpus=n)
    try:
        assert m.n_gpus == n
        g = sbr.fig5_grid(500).subset(np.arange(0, 500, 3))
        for ee in (0, 5):
            a = m.sweep_baseline(g, early_exit=ee)
            b = engine.sweep_baseline(g, early_exit=ee)
            for k in (*FIELDS, "status", "iters"):
                assert_same(a[k], b[k], f"n={n} {k} (early_exit={ee})")
        ph = m.host_phases()
        assert ph["slowest_rank_sweep"] > 0 and ph["host_copy_or_gather"] > 0
        with pytest.raises(Exception):
            m.sweep_baseline(g, flags=_lib.SBR_FLAG_RCCL_GATHER)
        h = sbr.hetero_config4(1024, 64).subset(np.arange(0, 1024, 97))
        a = m.sweep_hetero(h.betas, h.dist, h.eta, h.t_end, h.u, h.p, h.kappa, h.lam, h.x0)
        b = engine.sweep_hetero(h.betas, h.dist, h.eta, h.t_end, h.u, h.p, h.kappa, h.lam, h.x0)
        for k in ("xi", "aw_max", "tol", "status", "iters", "tau_in_unc", "tau_out_unc"):
            assert_same(a[k], b[k], f"n={n} hetero {k}")
        beta = 1.0 / sbr.julia_range("0.0001", "1", 30)
        u = sbr.julia_range("0.001", "1", 20)
        a = m.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
        b = engine.sweep_interest(beta, 15.0, 30.0, u, 0.5, 0.6, 0.01, 0.06, 0.1)
        for k in (*FIELDS, "status", "iters", "rk_steps"):
            assert_same(a[k], b[k], f"n={n} interest {k}")
        bs = 1.0 / sbr.julia_range("0.01", "2", 512)[[0, 100, 200, 511]]
        us = sbr.julia_range("0.001", "1", 512)[[10, 300]]
        a = m.sweep_social(bs, 30.0 / 0.9, us, 0.99, 0.25, 0.25, max_iter=3)
        b = engine.sweep_social(bs, 30.0 / 0.9, us, 0.99, 0.25, 0.25, max_iter=3)
        for k in (*FIELDS, "status", "iters", "fp_iters", "rk_steps"):
            assert_same(a[k], b[k], f"n={n} social {k}")
    finally:
        m.close()
