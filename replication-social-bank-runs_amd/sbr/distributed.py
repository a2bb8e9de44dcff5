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

from .grids import BaselineGrid

FLOAT_FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol")


def shard_columns(n_cols: int, world: int, rank: int) -> np.ndarray:
    """Interleaved column ownership: rank r gets r, r+world, r+2·world, …"""
    return np.arange(rank, n_cols, world)


def max_shard(n_cols: int, world: int) -> int:
    return (n_cols + world - 1) // world


def gather_columns(local: dict, n_cols: int, n_u: int, world: int, rank: int, device, root: int = 0):
    """Gather per-rank column blocks (numpy [n_local, n_u]) to `root` and put
    them back in global column order.  Returns the full dict on root, None
    elsewhere.  Each field travels as one padded tensor per rank (RCCL/gloo gather)."""
    m = max_shard(n_cols, world)
    out = {} if rank == root else None
    for f in (*FLOAT_FIELDS, "status"):
        if f not in local:
            continue
        a = np.asarray(local[f])
        dt = torch.float64 if f != "status" else torch.int32
        pad = np.zeros((m, n_u), dtype=np.float64 if f != "status" else np.int32)
        src = a.view(np.int32) if f == "status" else a
        pad[: a.shape[0]] = src
        t = torch.from_numpy(pad).to(device)
        bufs = [torch.empty_like(t) for _ in range(world)] if rank == root else None
        dist.gather(t, bufs, dst=root)
        if rank == root:
            full = np.empty((n_cols, n_u), dtype=pad.dtype)
            for r in range(world):
                cols = shard_columns(n_cols, world, r)
                full[cols] = bufs[r].cpu().numpy()[: len(cols)]
            out[f] = full.view(np.uint32) if f == "status" else full
    return out


def sweep_baseline_sharded(grid: BaselineGrid, compute: Callable[[BaselineGrid], dict] | None = None,
                           device=None, root: int = 0):
    """Shard `grid` over the ranks of the default process group, solve each
    shard with `compute` (default: this rank's GPU through libsbr), gather to root."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    if compute is None:
        from .engine import default_engine

        eng = default_engine()
        compute = lambda g: eng.sweep_baseline(g)  # noqa: E731
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    cols = shard_columns(len(grid.beta), world, rank)
    local = compute(grid.subset(cols)) if len(cols) else {f: np.zeros((0, len(grid.u))) for f in FLOAT_FIELDS}
    if "status" not in local:
        local["status"] = np.zeros((len(cols), len(grid.u)), np.uint32)
    if world == 1:
        return local
    return gather_columns(local, len(grid.beta), len(grid.u), world, rank, device, root)
