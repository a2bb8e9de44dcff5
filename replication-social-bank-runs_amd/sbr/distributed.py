"""Multi-GPU sharding of the parameter-grid sweep (one process per GPU).

Every grid point is independent, so a sweep shards over β
columns with no data-path collective: rank r owns the columns r, r+N, r+2N, …
(interleaved, so the β-dependent cost — knot count, run-region length — is
balanced).  The only exchange is the final gather of the result tensor to the
root over RCCL (xGMI), as equal-size padded blocks.

The per-rank compute is a callable so the same code path is exercised by the
CPU `gloo` tests (with the oracle as the compute) and by the GPU product
(libsbr through ``Engine``).
"""
from __future__ import annotations

from typing import Callable

import numpy as np
import torch
import torch.distributed as dist

from .grids import BaselineGrid, HeteroGrid, julia_range

FLOAT_FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")
INT_FIELDS = ("status", "iters", "fp_iters")


def shard_columns(n_cols: int, world: int, rank: int) -> np.ndarray:
    """Interleaved column ownership: rank r gets r, r+world, r+2·world, …"""
    return np.arange(rank, n_cols, world)


def max_shard(n_cols: int, world: int) -> int:
    return (n_cols + world - 1) // world


def gather_columns(local: dict, n_cols: int, n_u: int, world: int, rank: int, device, root: int = 0):
    """Gather per-rank column blocks (numpy [n_local, n_u]) to `root` and put
    them back in global column order.  Returns the full dict on root, None
    elsewhere.  Each field travels as one padded tensor per rank (RCCL/gloo gather);
    floats as float64, status / iteration counts as int32."""
    m = max_shard(n_cols, world)
    out = {} if rank == root else None
    for f in (*FLOAT_FIELDS, *INT_FIELDS):
        if f not in local:
            continue
        a = np.asarray(local[f])
        if a.ndim != 2:  # per-group hetero buffers [n, n_u, K] stay on the ranks
            continue
        is_int = f in INT_FIELDS
        pad = np.zeros((m, n_u), dtype=np.int32 if is_int else np.float64)
        pad[: a.shape[0]] = a.view(np.int32) if is_int else a
        t = torch.from_numpy(pad).to(device)
        bufs = [torch.empty_like(t) for _ in range(world)] if rank == root else None
        dist.gather(t, bufs, dst=root)
        if rank == root:
            full = np.empty((n_cols, n_u), dtype=pad.dtype)
            for r in range(world):
                cols = shard_columns(n_cols, world, r)
                full[cols] = bufs[r].cpu().numpy()[: len(cols)]
            out[f] = full.view(a.dtype) if is_int else full
    return out


def _world_rank():
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    return world, rank


def _device(device):
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    return device


def sweep_baseline_sharded(grid: BaselineGrid, compute: Callable[[BaselineGrid], dict] | None = None,
                           device=None, root: int = 0):
    """Shard `grid` over the ranks of the default process group, solve each
    shard with `compute` (default: this rank's GPU through libsbr), gather to root."""
    world, rank = _world_rank()
    if compute is None:
        from .engine import default_engine

        eng = default_engine()
        compute = lambda g: eng.sweep_baseline(g)  # noqa: E731
    device = _device(device)
    cols = shard_columns(len(grid.beta), world, rank)
    local = compute(grid.subset(cols)) if len(cols) else {f: np.zeros((0, len(grid.u))) for f in FLOAT_FIELDS}
    if "status" not in local:
        local["status"] = np.zeros((len(cols), len(grid.u)), np.uint32)
    if world == 1:
        return local
    return gather_columns(local, len(grid.beta), len(grid.u), world, rank, device, root)


def sweep_hetero_sharded(grid: HeteroGrid, compute: Callable[[HeteroGrid], dict] | None = None, device=None,
                         root: int = 0):
    """Heterogeneity sweep sharded over parameter columns like the baseline
    (rank r owns columns r, r+N, …); per-group buffers stay on the ranks."""
    world, rank = _world_rank()
    if compute is None:
        from .engine import default_engine

        eng = default_engine()
        compute = lambda g: eng.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam,  # noqa: E731
                                             g.x0, with_groups=False)
    cols = shard_columns(grid.betas.shape[0], world, rank)
    local = compute(grid.subset(cols))
    if world == 1:
        return local
    return gather_columns(local, grid.betas.shape[0], len(grid.u), world, rank, _device(device), root)


def sweep_social_sharded(beta, eta, u, p, kappa, lam, cmp=None, x0=1e-4, tol=1e-4, max_iter=500,
                         compute: Callable[..., dict] | None = None, device=None, root: int = 0):
    """Social-learning sweep (social_learning_solver.jl:63-263) sharded over β
    columns; every point is an independent fixed point, so the only exchange is
    the gather of the results.  compute(beta, eta, u, cmp) solves one shard."""
    world, rank = _world_rank()
    beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
    eta = np.ascontiguousarray(np.broadcast_to(eta, beta.shape), np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    if cmp is None:
        cmp = np.stack([julia_range(0.0, float(e), 1000) for e in eta])
    cmp = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(cmp), (len(beta), np.atleast_2d(cmp).shape[1])))
    if compute is None:
        from .engine import default_engine

        eng = default_engine()
        compute = lambda b, e, uu, c: eng.sweep_social(b, e, uu, p, kappa, lam, cmp=c, x0=x0, tol=tol,  # noqa: E731
                                                       max_iter=max_iter)
    cols = shard_columns(len(beta), world, rank)
    local = compute(beta[cols], eta[cols], u, cmp[cols])
    if world == 1:
        return local
    return gather_columns(local, len(beta), len(u), world, rank, _device(device), root)


def sweep_interest_sharded(beta, eta, t_end, u, p, kappa, lam, r, delta, x0=1e-4,
                           compute: Callable[..., dict] | None = None, device=None, root: int = 0):
    """Interest-rate sweep (interest_rate_solver.jl:51-150) sharded over β columns:
    every point's value function and equilibrium are independent, so the only
    exchange is the result gather.  compute(beta, eta, t_end, u) solves one shard."""
    world, rank = _world_rank()
    beta = np.ascontiguousarray(np.atleast_1d(beta), np.float64)
    eta = np.ascontiguousarray(np.broadcast_to(eta, beta.shape), np.float64)
    t_end = np.ascontiguousarray(np.broadcast_to(t_end, beta.shape), np.float64)
    u = np.ascontiguousarray(np.atleast_1d(u), np.float64)
    if compute is None:
        from .engine import default_engine

        eng = default_engine()
        compute = lambda b, e, t, uu: eng.sweep_interest(b, e, t, uu, p, kappa, lam, r, delta, x0=x0)  # noqa: E731
    cols = shard_columns(len(beta), world, rank)
    local = compute(beta[cols], eta[cols], t_end[cols], u)
    if world == 1:
        return local
    return gather_columns(local, len(beta), len(u), world, rank, _device(device), root)


class StepCollector:
    """Collect the full result SoA of every step of a weak-scaled sweep, each step's grid on
    one rank: step k — every rank's column shard of it — lands on rank k mod N (the
    grid's "root").  A window of up to N consecutive steps k0 … k0+m−1 with distinct roots
    is collected by one all-to-all per field (rank q sends its shard of step k to rank
    k mod N), so every xGMI link carries its share in both directions.  A gather of every
    step to rank 0 is capped by rank 0's inbound links instead: at config 3 each rank
    produces ≈201 MB of results per ≈1.9 ms step, and 7 of those per step exceed the
    ≈0.54 TB/s that one MI355X's 7 links take in.

    fields: {name: tensor [n_steps, n_pts]} (this rank's shard of every step, one row per
    step; any dtype the backend moves).  After collect(k0, m), rank (k mod N) holds, for
    every field, ranks 0…N−1's shards of step k in ``recv[name][q]`` (q = source rank).
    """

    def __init__(self, fields: dict, world: int, rank: int):
        self.fields, self.world, self.rank = fields, world, rank
        self.n_pts = {f: t.shape[1] for f, t in fields.items()}
        self.recv = {f: torch.empty(world, t.shape[1], dtype=t.dtype, device=t.device) for f, t in fields.items()}
        self._empty = {f: torch.empty(0, dtype=t.dtype, device=t.device) for f, t in fields.items()}
        self.last_roots: list[int] = []

    def window_roots(self, k0: int, m: int) -> list[int]:
        roots = [(k0 + i) % self.world for i in range(m)]
        if m > self.world or len(set(roots)) != m:
            raise ValueError("a window holds at most one step per root")
        return roots

    def collect(self, k0: int, m: int = 1, row0: int | None = None) -> None:
        """Steps k0 … k0+m−1 are complete on every rank; move them to their roots.  Their
        shards are rows row0 … row0+m−1 of each field (default row0 = k0; a caller that
        reuses one row per step passes row0 = 0, m = 1).  The window must be contiguous in
        root order (k0 mod N + m ≤ N), so that the shards to send are one contiguous slice
        of each field."""
        roots = self.window_roots(k0, m)
        first = roots[0]
        if first + m > self.world:
            raise ValueError("window wraps past rank N-1: split it")
        self.last_roots = roots
        r0 = k0 if row0 is None else row0
        for f, t in self.fields.items():
            n = self.n_pts[f]
            src = t[r0:r0 + m].reshape(-1)
            in_splits = [n if first <= r < first + m else 0 for r in range(self.world)]
            is_root = first <= self.rank < first + m
            out = self.recv[f].view(-1) if is_root else self._empty[f]
            dist.all_to_all_single(out, src, [n] * self.world if is_root else [0] * self.world, in_splits)

    def windows(self, n_steps: int):
        """(k0, m) windows covering steps 0 … n_steps−1, each within one round of N roots."""
        k = 0
        while k < n_steps:
            m = min(self.world - k % self.world, n_steps - k)
            yield k, m
            k += m
