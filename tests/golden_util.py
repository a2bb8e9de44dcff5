"""Helpers that turn oracle outputs into the quantities the reference's
figures plot (so they can be compared with tests/golden/)."""
import numpy as np


def interp(knots, vals, x):
    """Interpolations.jl gridded Linear (same formula as the oracle)."""
    knots = np.asarray(knots)
    vals = np.asarray(vals)
    x = np.asarray(x, np.float64)
    assert np.all((x >= knots[0]) & (x <= knots[-1])), "BoundsError"
    j = np.clip(np.searchsorted(knots, x, side="right") - 1, 0, len(knots) - 2)
    d = (x - knots[j]) / (knots[j + 1] - knots[j])
    return vals[j] * (1.0 - d) + vals[j + 1] * d


def aw_paths(xi, tin, tout, tau, t, G):
    """get_AW (solver.jl:495-532) on the HR grid tau: AW_cum, AW_OUT, AW_IN."""
    ic = xi if tin >= xi else tin
    oc = xi if tout > xi else tout
    a = (tau - xi) + ic
    b = (tau - xi) + oc
    awin = np.where(a >= 0, interp(t, G, np.where(a > 0, a, 0.0)), 0.0)
    awout = np.where(b >= 0, interp(t, G, np.where(b > 0, b, 0.0)), 0.0)
    return (awout - awin) + interp(t, G, 0.0), awout, awin


def viridis_level(rgb, palette):
    """Position in [0, 1] (0 = data min) of colours on GR's interpolated
    256-entry palette (palette[0] = top of the colourbar = data max)."""
    pal = palette[::-1].astype(np.float64)  # pal[0] = min
    seg_a, seg_b = pal[:-1], pal[1:]
    d = seg_b - seg_a
    c = rgb.astype(np.float64)[:, None, :]
    w = np.clip(((c - seg_a) * d).sum(-1) / np.maximum((d * d).sum(-1), 1e-12), 0, 1)
    proj = seg_a + w[..., None] * d
    dist = ((c - proj) ** 2).sum(-1)
    k = dist.argmin(1)
    return (k + w[np.arange(len(k)), k]) / 255.0, dist.min(1)
