"""Figure regeneration from saved sweeps — presentation
only, never on the hot path.  Mirrors the two sweep figures of
scripts/1_baseline.jl: the Fig 5 β-u heatmap of max aggregate withdrawals
(:195-200, :278-284: viridis, NaN = no run, x = average meeting time 1/β) and
the Fig 4 comparative statics in u (:170-192)."""
from __future__ import annotations

import numpy as np


def _plt():
    import matplotlib

    matplotlib.use("Agg")
    import matplotlib.pyplot as plt

    return plt


def heatmap_fig5(arrays: dict, out_path, title: str = "Max aggregate withdrawals"):
    """Heatmap of max_AW_matrix over (1/β, u) as in comp_stat_cross_heatmap_AW.pdf."""
    plt = _plt()
    beta = arrays["axis_beta"]
    u = arrays["axis_u"]
    m = np.asarray(arrays["aw_max"]).T  # [n_u, n_β]
    fig, ax = plt.subplots(figsize=(6, 4.5))
    im = ax.imshow(np.ma.masked_invalid(m), origin="lower", aspect="auto", cmap="viridis", alpha=0.8,
                   extent=[float(1 / beta[0]), float(1 / beta[-1]), float(u[0]), float(u[-1])])
    ax.set_xlabel("average meeting time 1/β")
    ax.set_ylabel("u")
    ax.set_title(title)
    fig.colorbar(im, ax=ax)
    fig.savefig(out_path, bbox_inches="tight")
    plt.close(fig)
    return out_path


def comparative_statics_u(arrays: dict, out_path, column: int = 0):
    """AW_max(u) and ξ(u) of one β column (Fig 4 panels a/b, comp_stat_u_panel_*.pdf)."""
    plt = _plt()
    u = arrays["axis_u"]
    aw = np.asarray(arrays["aw_max"])[column]
    xi = np.asarray(arrays["xi"])[column]
    fig, (a, b) = plt.subplots(1, 2, figsize=(9, 3.5))
    a.plot(u, aw)
    a.set_xlabel("u")
    a.set_ylabel("max AW")
    b.plot(u, xi)
    b.set_xlabel("u")
    b.set_ylabel("ξ*")
    fig.savefig(out_path, bbox_inches="tight")
    plt.close(fig)
    return out_path
