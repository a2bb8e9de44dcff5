"""The N>1 path on CPU: world_size-2 (and 3) `gloo` process groups shard a
grid over β columns, solve each shard (the oracle stands in for the per-rank
GPU), and gather to rank 0 — the result equals the single-process sweep."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import sbr
from sbr import distributed as D

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "replication-social-bank-runs_amd"))
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    grid = sbr.fig5_grid(37, n_u=60)

    def compute(g):
        return O.sweep_baseline(g.beta, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0)

    res = D.sweep_baseline_sharded(grid, compute=compute, device="cpu")
    if rank == 0:
        np.savez(out_path, **res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_sweep_equals_single_process(tmp_path, oracle, world):
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    grid = sbr.fig5_grid(37, n_u=60)
    ref = oracle.sweep_baseline(grid.beta, grid.eta, grid.t_end, grid.u, grid.p, grid.kappa, grid.lam, grid.x0)
    for f in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol"):
        a, b = got[f], ref[f]
        assert a.shape == b.shape
        assert np.all((a == b) | (np.isnan(a) & np.isnan(b))), f
    assert np.array_equal(got["status"], ref["status"])


def _worker_ext(rank, world, port, out_path):
    """Social and hetero sweeps sharded the same way (oracle as per-rank compute)."""
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "replication-social-bank-runs_amd"))
    import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    beta, u, eta = _social_axes()
    soc = D.sweep_social_sharded(beta, eta, u, 0.99, 0.25, 0.25, max_iter=3, device="cpu",
                                 compute=lambda b, e, uu, c: O.sweep_social(b, e, uu, 0.99, 0.25, 0.25, c,
                                                                            max_iter=3))
    hg = sbr.hetero_config4(5, 7, K=2)
    het = D.sweep_hetero_sharded(hg, device="cpu", compute=lambda g: O.sweep_hetero(
        g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0))
    ib, iu = _interest_axes()
    itr = D.sweep_interest_sharded(ib, 15.0, 30.0, iu, 0.5, 0.6, 0.01, 0.06, 0.1, device="cpu",
                                   compute=lambda b, e, t, uu: O.sweep_interest(b, e, t, uu, 0.5, 0.6, 0.01, 0.06,
                                                                                0.1))
    if rank == 0:
        np.savez(out_path, **{"s_" + k: v for k, v in soc.items()}, **{"h_" + k: v for k, v in het.items()},
                 **{"i_" + k: v for k, v in itr.items()})
    dist.barrier()
    dist.destroy_process_group()


def _interest_axes():
    return 1.0 / sbr.julia_range("0.0001", "1", 500)[[0, 60, 250, 499, 120]], sbr.julia_range("0.001", "1", 500)[::60]


def _social_axes():
    beta = 1.0 / sbr.julia_range("0.01", "2", 512)[[0, 100, 300, 511, 200]]
    u = sbr.julia_range("0.001", "1", 512)[[40, 300]]
    return beta, u, 30.0 / 0.9


def test_sharded_social_hetero_interest_equal_single_process(tmp_path, oracle):
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker_ext, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    beta, u, eta = _social_axes()
    ref = oracle.sweep_social(beta, eta, u, 0.99, 0.25, 0.25, sbr.julia_range(0.0, eta, 1000), max_iter=3)
    for f in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters", "fp_iters"):
        a, b = got["s_" + f], ref[f]
        assert a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), f
    ib, iu = _interest_axes()
    iref = oracle.sweep_interest(ib, 15.0, 30.0, iu, 0.5, 0.6, 0.01, 0.06, 0.1)
    for f in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters"):
        a, b = got["i_" + f], iref[f]
        assert a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), f
    hg = sbr.hetero_config4(5, 7, K=2)
    href = oracle.sweep_hetero(hg.betas, hg.dist, hg.eta, hg.t_end, hg.u, hg.p, hg.kappa, hg.lam, hg.x0)
    for f in ("xi", "aw_max", "tol", "status", "iters"):
        a, b = got["h_" + f], href[f]
        assert a.shape == b.shape and np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), f


def test_shard_columns_partition():
    for n, w in ((2048, 8), (37, 3), (5, 8)):
        parts = [D.shard_columns(n, w, r) for r in range(w)]
        allc = np.sort(np.concatenate(parts))
        assert np.array_equal(allc, np.arange(n))
        assert max(len(p) for p in parts) == D.max_shard(n, w)


def _worker_collect(rank, world, port, out_path):
    """Every step's full result SoA on its root (rank k mod N) via StepCollector."""
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.join(REPO, "replication-social-bank-runs_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_steps, n_pts = 7, 11
    # rank r's shard of step k: values that encode (field, step, rank, point)
    base = torch.arange(n_steps * n_pts, dtype=torch.float64).view(n_steps, n_pts)
    fields = {"xi": base + 1000.0 * rank, "status": (base * 3 + rank).to(torch.int32),
              "rk_steps": (base * 7 + 100000 * rank).to(torch.int64)}
    col = D.StepCollector(fields, world, rank)
    got = {}
    for k0, m in col.windows(n_steps):
        col.collect(k0, m)
        for i, root in enumerate(col.last_roots):
            if root == rank:
                got[k0 + i] = {f: col.recv[f].clone().numpy() for f in fields}
    np.savez(out_path + f".{rank}.npz", **{f"{k}_{f}": v for k, d in got.items() for f, v in d.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_step_collector_round_robin_roots(tmp_path, world):
    out = str(tmp_path / "col")
    mp.spawn(_worker_collect, args=(world, _free_port(), out), nprocs=world, join=True)
    n_steps, n_pts = 7, 11
    base = np.arange(n_steps * n_pts, dtype=np.float64).reshape(n_steps, n_pts)
    seen = set()
    for r in range(world):
        d = np.load(out + f".{r}.npz")
        for key in d.files:
            k, f = key.split("_", 1)
            k = int(k)
            assert k % world == r  # step k is collected on rank k mod N
            seen.add(k)
            for q in range(world):
                exp = {"xi": base[k] + 1000.0 * q, "status": (base[k] * 3 + q).astype(np.int32),
                       "rk_steps": (base[k] * 7 + 100000 * q).astype(np.int64)}[f]
                assert np.array_equal(d[key][q], exp), (k, f, q)
    assert seen == set(range(n_steps))
