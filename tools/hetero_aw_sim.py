"""Operation counts of AW_max strategies for the heterogeneity kernel, simulated on the CPU from
the oracle's config-4 columns (design aid for equilibrium_hetero_kernel's AW phase; not a test).

For sampled run points it counts what each strategy issues per point:
  * `bnb`    — the kernel's branch and bound (pass 1 best 256/64/8 descent + pass 2 sweep);
              a bound call costs 2K bracket searches + 2K G gathers;
  * `coarse` — the same tree, 256- and 64-knot bounds from ω = Σ_k dist_k G_k (2 searches +
              2 gathers), 8-knot bounds per group;
  * `walk`   — outward scan from pass 1's best knot: right of the last exact knot i the bound
              ω[j+2] − IN(i), left of it OUT(i) − ω[bracket(a_min(j))]; each jump is one ω
              gallop + one t gallop + an exact evaluation.
Exact evaluations cost 2K lerps (4K G gathers) with walker brackets.
Prints one JSON line with per-point means."""
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
from oracle import oracle  # noqa: E402
import sbr  # noqa: E402


def ssl(t, x):
    return np.clip(np.searchsorted(t, x, side="right") - 1, 0, len(t) - 2)


def lerp(t, g, j, x):
    d = (x - t[j]) / (t[j + 1] - t[j])
    return g[j] * (1 - d) + g[j + 1] * d


def aw_parts(t, G, xi, icc, occ, dist):
    n, K = G.shape
    OUT = np.zeros(n)
    IN = np.zeros(n)
    for k in range(K):
        av = (t - xi) + icc[k]
        bv = (t - xi) + occ[k]
        xa, xb = np.maximum(av, 0), np.maximum(bv, 0)
        gi = np.where(av >= 0, lerp(t, G[:, k], ssl(t, xa), xa), 0.0)
        go = np.where(bv >= 0, lerp(t, G[:, k], ssl(t, xb), xb), 0.0)
        OUT += dist[k] * go
        IN += dist[k] * gi
    return OUT, IN


def drawdown_env(G, dist):
    d = np.diff(G, axis=0)
    env = 0.0
    for k in range(G.shape[1]):
        dec = -d[:, k][d[:, k] < 0]
        env += dist[k] * 2.0 * (len(dec) * (dec.max() if len(dec) else 0.0))
    return env


class Point:
    def __init__(self, t, G, dist, xi, tin, tout, env):
        self.t, self.G, self.dist, self.xi, self.env = t, G, dist, xi, env
        self.n, self.K = G.shape
        self.icc, self.occ = np.minimum(tin, xi), np.minimum(tout, xi)
        self.OUT, self.IN = aw_parts(t, G, xi, self.icc, self.occ, dist)
        self.aw = self.OUT - self.IN
        self.om = G @ dist
        self.sep = bool(np.all(t[2:] - t[:-2] > 1e-15 * t[-1]))

    def ub_fine(self, i0, i1):
        t, G, n = self.t, self.G, self.n
        s = 0.0
        for k in range(self.K):
            bv = (t[i1] - self.xi) + self.occ[k]
            if self.sep and self.occ[k] == self.xi:
                hi = max(G[min(i1 + 2, n - 1), k], 0.0)
            elif bv >= 0:
                hi = max(G[min(ssl(t, bv) + 1, n - 1), k], 0.0)
            else:
                hi = 0.0
            av = (t[i0] - self.xi) + self.icc[k]
            lo = G[ssl(t, av), k] if av >= 0 else min(G[0, k], 0.0)
            s += self.dist[k] * (hi - lo)
        return s + 1e-14 + self.env

    def ub_coarse(self, i0, i1):
        t, n, om = self.t, self.n, self.om
        bmax = (t[i1] - self.xi) + self.occ.max()
        hi = om[min(ssl(t, bmax) + 1, n - 1)] if bmax >= 0 else 0.0
        amin = (t[i0] - self.xi) + self.icc.min()
        lo = om[ssl(t, amin)] if amin >= 0 else 0.0
        return hi - lo + 1e-14 + self.env


def tree(P, coarse_levels):
    """pass 1 + pass 2 of the kernel's branch and bound; returns (fine calls, coarse calls, evals)."""
    n = P.n
    cnt = dict(fine=0, coarse=0, evals=0)

    def ub(i0, i1, w):
        if w in coarse_levels:
            cnt["coarse"] += 1
            return P.ub_coarse(i0, i1)
        cnt["fine"] += 1
        return P.ub_fine(i0, i1)

    end = lambda i0, w: min(i0 + w, n)
    best, bu = 0, -np.inf
    for i0 in range(0, n, 256):
        u = ub(i0, end(i0, 256) - 1, 256)
        if not u <= bu:
            bu, best = u, i0
    bb, bu = best, -np.inf
    for i0 in range(best, end(best, 256), 64):
        u = ub(i0, end(i0, 64) - 1, 64)
        if not u <= bu:
            bu, bb = u, i0
    b8, bu = bb, -np.inf
    for i0 in range(bb, end(bb, 64), 8):
        u = ub(i0, end(i0, 8) - 1, 8)
        if not u <= bu:
            bu, b8 = u, i0
    mx = P.aw[b8:end(b8, 8)].max()
    cnt["evals"] += end(b8, 8) - b8
    for s0 in range(0, n, 256):
        se = end(s0, 256)
        if ub(s0, se - 1, 256) <= mx:
            continue
        for k0 in range(s0, se, 64):
            ke = end(k0, 64)
            if ub(k0, ke - 1, 64) <= mx:
                continue
            for i0 in range(k0, ke, 8):
                ie = end(i0, 8)
                if i0 == b8 or ub(i0, ie - 1, 8) <= mx:
                    continue
                mx = max(mx, P.aw[i0:ie].max())
                cnt["evals"] += ie - i0
    assert mx == P.aw.max(), (mx, P.aw.max())
    return cnt, b8


def walk(P, start):
    """outward scan from knot `start`; returns (jumps right, jumps left)."""
    t, n, om, xi = P.t, P.n, P.om, P.xi
    omax, imin = P.occ.max(), P.icc.min()
    marg = 1e-14 + P.env
    mx = P.aw[start]
    jr = jl = 0
    i = start
    while True:  # right
        thr = mx + P.IN[i] + marg           # dismiss j with ω[j+2] <= thr (b_k(t_j) <= t_j + ulp)
        q = int(np.searchsorted(om, thr, side="right"))  # first index with ω > thr (ω nondecreasing up to env)
        j = max(i + 1, q - 2)
        if j >= n:
            break
        # also j must satisfy b_max(t_j) bracket: with occ_k < ξ the bound ω[j+2] is loose but valid
        i = j
        jr += 1
        mx = max(mx, P.aw[i])
    i = start
    while True:  # left
        thr = P.OUT[i] - mx + marg          # dismiss j with ω[bracket(a_min(t_j))] >= thr
        if thr <= 0:
            break
        q = int(np.searchsorted(om, thr, side="left"))   # first ω >= thr
        if q >= n:
            j = i - 1
        else:
            # a_min(t_j) >= t[q]  ⇔  t_j >= t[q] + ξ − icc_min: those are dismissed
            lim = t[q] + xi - imin
            j = min(i - 1, int(np.searchsorted(t, lim, side="left")) - 1)
        if j < 0:
            break
        i = j
        jl += 1
        mx = max(mx, P.aw[i])
    assert mx == P.aw.max() or abs(mx - P.aw.max()) < 1e-15, (mx, P.aw.max())
    return jr, jl


def main(n_cols=6, n_pts=24, N=1024):
    g = sbr.hetero_config4(N, N, K=8)
    cols = np.linspace(0, N - 1, n_cols).astype(int)
    stats = dict(bnb_fine=[], cfine=[], ccoarse=[], bnb_evals=[], c_evals=[], walk_r=[], walk_l=[], n=[])
    for c in cols:
        t, G, _ = oracle.learn_hetero(g.betas[c], g.dist, float(g.t_end[c]))
        o = oracle.hetero_equilibrium_knots(t, G, g.betas[c], g.dist, float(g.eta[c]), float(g.t_end[c]), g.u, g.p,
                                            g.kappa, g.lam)
        run = np.nonzero(o["status"] & 1)[0]
        if len(run) == 0:
            continue
        env = drawdown_env(G, g.dist)
        for j in run[np.linspace(0, len(run) - 1, min(n_pts, len(run))).astype(int)]:
            P = Point(t, G, g.dist, o["xi"][j], o["tau_in_unc"][j], o["tau_out_unc"][j], env)
            a, b8 = tree(P, ())
            cc, _ = tree(P, (256, 64))
            jr, jl = walk(P, b8 + int(np.argmax(P.aw[b8:b8 + 8])))
            stats["bnb_fine"].append(a["fine"]); stats["bnb_evals"].append(a["evals"])
            stats["cfine"].append(cc["fine"]); stats["ccoarse"].append(cc["coarse"]); stats["c_evals"].append(cc["evals"])
            stats["walk_r"].append(jr); stats["walk_l"].append(jl); stats["n"].append(P.n)
    print(json.dumps({k: float(np.mean(v)) for k, v in stats.items()} | {"points": len(stats["n"])}))


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
