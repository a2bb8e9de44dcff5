"""The n-device data movement of libsbr without GPUs.

sbr_init_multi sweeps deal grid columns cyclically over N GPUs, pack each rank's results
into one block, and return them into the caller's u-fastest arrays — each rank scattering
its own block (the default direct transport: every GPU's own PCIe link), or a gather of the
blocks to rank 0 and one scatter from there (SBR_FLAG_RCCL_GATHER) (csrc/sbr_shard.h, driven
by csrc/sbr_multi.hip with hipMemcpy2DAsync / RCCL).  sbr_shard_host_run runs that same code
with a host loopback transport and a caller-supplied per-rank sweep:
here the CPU oracle on exactly the columns the deal hands each rank.  At N = 2, 3, 8 —
including n_col < N and n_col % N != 0 — the scattered arrays must equal the oracle's
single-grid sweep bit for bit, for the baseline fields (f64 and u32/i32) and the hetero
per-group buffers (per_pt = K)."""
import ctypes

import numpy as np
import pytest

import sbr
from sbr import _lib

CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64),
                      ctypes.POINTER(ctypes.c_void_p))


def _host_run(n_ranks, n_col, n_u, specs, per_rank, rccl_gather=0):
    """specs: [(name, dtype, per_pt)]; per_rank(col_ids) -> {name: array [n, n_u(, per_pt)]}."""
    L = _lib.load()
    L.sbr_shard_host_run.restype = ctypes.c_int
    L.sbr_shard_host_run.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, CB, ctypes.c_void_p, ctypes.c_int32]
    out = {n: np.full(n_col * n_u * pp, 0xAB, dtype=np.dtype(dt)).view(dt) for n, dt, pp in specs}
    esz = np.array([np.dtype(dt).itemsize for _, dt, _ in specs], np.int64)
    per_pt = np.array([pp for _, _, pp in specs], np.int64)
    ptrs = (ctypes.c_void_p * len(specs))(*[out[n].ctypes.data for n, _, _ in specs])
    seen = []

    def compute(user, rank, nc, ids, fields):
        cols = np.array([ids[i] for i in range(nc)], np.int64)
        seen.append((rank, cols))
        res = per_rank(cols)
        for f, (n, dt, pp) in enumerate(specs):
            a = np.ascontiguousarray(res[n], dtype=dt).reshape(-1)
            assert a.size == nc * n_u * pp
            ctypes.memmove(fields[f], a.ctypes.data, a.nbytes)
        return 0

    cb = CB(compute)
    rc = L.sbr_shard_host_run(n_ranks, n_col, n_u, len(specs), esz.ctypes.data, per_pt.ctypes.data, ptrs, cb, None,
                              rccl_gather)
    assert rc == 0
    return out, seen


BASE_SPECS = [("xi", np.float64, 1), ("tau_in_unc", np.float64, 1), ("tau_out_unc", np.float64, 1),
              ("aw_max", np.float64, 1), ("tol", np.float64, 1), ("status", np.uint32, 1), ("iters", np.int32, 1)]


@pytest.fixture(scope="module")
def small_grid():
    g = sbr.fig5_grid(500)
    return g.subset(np.arange(3, 500, 37))  # 14 β columns spanning the Fig 5 range


@pytest.fixture(scope="module")
def full_baseline(oracle, small_grid):
    g = small_grid
    u = g.u[::25]
    return u, oracle.sweep_baseline(g.beta, g.eta, g.t_end, u, g.p, g.kappa, g.lam, g.x0)


@pytest.mark.parametrize("transport", [0, 1], ids=["direct", "gather"])
@pytest.mark.parametrize("N", [1, 2, 3, 8, 20])
def test_shard_layout_baseline_equals_single_grid(oracle, small_grid, full_baseline, N, transport):
    g = small_grid
    u, ref = full_baseline
    nb, nu = len(g.beta), len(u)

    def per_rank(cols):
        return oracle.sweep_baseline(g.beta[cols], g.eta[cols], g.t_end[cols], u, g.p, g.kappa, g.lam, g.x0)

    out, seen = _host_run(N, nb, nu, BASE_SPECS, per_rank, transport)
    # the deal: rank r gets columns r, r+N, …; every column exactly once
    for rank, cols in seen:
        assert np.array_equal(cols, np.arange(rank, nb, N))
    assert sorted(np.concatenate([c for _, c in seen]).tolist()) == list(range(nb))
    assert len(seen) == min(N, nb)  # ranks without columns compute nothing
    for n, dt, _ in BASE_SPECS:
        a, b = out[n].reshape(nb, nu), ref[n]
        assert np.array_equal(a, b, equal_nan=np.dtype(dt).kind == "f"), (N, n)


@pytest.mark.parametrize("transport", [0, 1], ids=["direct", "gather"])
@pytest.mark.parametrize("N", [2, 3, 8, 20])
def test_shard_layout_hetero_per_group_fields(oracle, N, transport):
    g = sbr.hetero_config4(7, 6, K=2)  # 7 columns: 7 % 2, 7 % 3 != 0, 7 < 8
    K = len(g.dist)
    specs = [("xi", np.float64, 1), ("aw_max", np.float64, 1), ("tol", np.float64, 1), ("status", np.uint32, 1),
             ("iters", np.int32, 1), ("tau_in_unc", np.float64, K), ("tau_out_unc", np.float64, K)]
    nc, nu = len(g.eta), len(g.u)
    ref = oracle.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0)

    def per_rank(cols):
        return oracle.sweep_hetero(g.betas[cols], g.dist, g.eta[cols], g.t_end[cols], g.u, g.p, g.kappa, g.lam, g.x0)

    out, _ = _host_run(N, nc, nu, specs, per_rank, transport)
    for n, dt, pp in specs:
        a = out[n].reshape(nc, nu, pp) if pp > 1 else out[n].reshape(nc, nu)
        assert np.array_equal(a, ref[n], equal_nan=np.dtype(dt).kind == "f"), (N, n)


def test_shard_host_run_rejects_bad_arguments():
    L = _lib.load()
    L.sbr_shard_host_run.restype = ctypes.c_int
    L.sbr_shard_host_run.argtypes = [ctypes.c_int32, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_void_p, CB, ctypes.c_void_p, ctypes.c_int32]
    cb = CB(lambda *a: 0)
    one = np.ones(1, np.int64)
    buf = np.zeros(4)
    ptrs = (ctypes.c_void_p * 1)(buf.ctypes.data)
    assert L.sbr_shard_host_run(0, 2, 2, 1, one.ctypes.data, one.ctypes.data, ptrs, cb, None, 0) == _lib.SBR_EARG
    assert L.sbr_shard_host_run(2, 0, 2, 1, one.ctypes.data, one.ctypes.data, ptrs, cb, None, 0) == _lib.SBR_EARG
    zero = np.zeros(1, np.int64)
    assert L.sbr_shard_host_run(2, 2, 2, 1, zero.ctypes.data, one.ctypes.data, ptrs, cb, None, 0) == _lib.SBR_EARG
    # a failing rank's compute aborts the run with its code, before any gather
    bad = CB(lambda *a: -7)
    assert L.sbr_shard_host_run(2, 2, 2, 1, one.ctypes.data, one.ctypes.data, ptrs, bad, None, 0) == -7
