"""Sweep results on disk: the reference never persists
its sweep matrices (scripts/1_baseline.jl:274-284 only saves the figure), so a
figure cannot be regenerated or compared without re-solving.  Here a sweep is
one ``.npz`` (result fields as [n_β, n_u] arrays, u-fastest like the C ABI,
plus the parameter axes) with a JSON metadata block: the workload name, the
scalar parameters, the status-bit legend, and the engine version.  Loading uses
``numpy.load(allow_pickle=False)`` only.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from ._lib import STATUS

FORMAT = "sbr-sweep-v1"
_ARRAY_FIELDS = ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters", "fp_iters", "rk_steps")


def save_sweep(path, result: dict, *, beta=None, u=None, eta=None, t_end=None, params: dict | None = None,
               workload: str = "") -> Path:
    """Write ``result`` (dict of [n_β, n_u] arrays from Engine.sweep_*) and the
    grid axes to ``path`` (.npz).  ``params`` holds the scalars (p, κ, λ, x0, tol…)."""
    from . import __version__

    path = Path(path)
    arrays = {k: np.asarray(v) for k, v in result.items() if k in _ARRAY_FIELDS and v is not None}
    for name, ax in (("beta", beta), ("u", u), ("eta", eta), ("t_end", t_end)):
        if ax is not None:
            arrays["axis_" + name] = np.asarray(ax, np.float64)
    meta = {"format": FORMAT, "workload": workload, "params": params or {}, "status_bits": STATUS,
            "engine_version": __version__, "layout": "[n_beta, n_u], u fastest (max_AW_matrix[j, i] = aw_max[i, j])"}
    arrays["meta_json"] = np.frombuffer(json.dumps(meta, sort_keys=True).encode(), dtype=np.uint8)
    np.savez_compressed(path, **arrays)
    return path if path.suffix == ".npz" else path.with_suffix(path.suffix + ".npz")


def load_sweep(path) -> tuple[dict, dict]:
    """(arrays, metadata) of a file written by save_sweep."""
    with np.load(path, allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files if k != "meta_json"}
        meta = json.loads(bytes(z["meta_json"]).decode())
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not an {FORMAT} file")
    return arrays, meta


def max_aw_matrix(arrays: dict) -> np.ndarray:
    """The reference's max_AW_matrix (scripts/1_baseline.jl:213,254): [n_u, n_β],
    NaN where there is no run or the point was skipped."""
    return np.asarray(arrays["aw_max"]).T
