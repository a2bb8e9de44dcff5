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


def test_shard_columns_partition():
    for n, w in ((2048, 8), (37, 3), (5, 8)):
        parts = [D.shard_columns(n, w, r) for r in range(w)]
        allc = np.sort(np.concatenate(parts))
        assert np.array_equal(allc, np.arange(n))
        assert max(len(p) for p in parts) == D.max_shard(n, w)
