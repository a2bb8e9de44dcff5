"""Counts aw_scan's exact AW evaluations per run point (csrc/sbr_baseline.hip) on the oracle's
knots of config-3 columns, for the shipped bounds and a variant, and checks that every variant's
maximum equals the exhaustive maximum bit for bit.  Test infrastructure / design tool (CPU)."""
import bisect
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "oracle"), str(REPO / "replication-social-bank-runs_amd")]
import oracle as O  # noqa: E402
import sbr  # noqa: E402


def ssl(T, x, lo=0, hi=None):
    hi = len(T) - 1 if hi is None else hi
    j = bisect.bisect_right(T, x, lo, hi + 1) - 1
    return max(j, lo)


def first_ge_down(key, hi, x):
    top, lo, step = hi, hi - 1, 1
    while lo >= 0 and key(lo) >= x:
        top = lo
        step <<= 1
        lo = top - step
    lo = max(lo, -1)
    while top - lo > 1:
        mid = (lo + top) >> 1
        if key(mid) >= x:
            top = mid
        else:
            lo = mid
    return top


def aw_scan(T, G, n, ntau, nle, ETA, xi, icc, occ, G0, dd, c, koff, variant):
    M = 1e-14 + 4.0 * dd
    tau = lambda i: T[i] if i < nle else ETA  # noqa: E731
    av_of = lambda i: (tau(i) - xi) + icc  # noqa: E731
    st = dict(ka=0, ta0=0., ta1=0., ga0=0., ga1=0., awin=0., awout=0., nev=0, mx=-np.inf, trips=0)
    own_ok = occ == xi

    def in_own(i):
        """b_i = (t_i − ξ) + ξ is t_i exactly (Sterbenz: t_i in [ξ/2, 2ξ])"""
        return own_ok and i < nle and 0.5 * xi <= T[i] <= 2.0 * xi

    def koff_of(i):
        return 0 if (variant == 2 and in_own(i)) else koff

    def seek(x):
        k = min(ssl(T, x), n - 2)
        st.update(ka=k, ta0=T[k], ta1=T[k + 1], ga0=G[k], ga1=G[k + 1])

    def fwd(x):
        while st["ka"] < n - 2 and st["ta1"] <= x:
            k = st["ka"] + 1
            st.update(ka=k, ta0=st["ta1"], ga0=st["ga1"], ta1=T[k + 1], ga1=G[k + 1])

    def bwd(x):
        while st["ka"] > 0 and st["ta0"] > x:
            k = st["ka"] - 1
            st.update(ka=k, ta1=st["ta0"], ga1=st["ga0"], ta0=T[k], ga0=G[k])

    def exact(i, av, xa):
        ti = tau(i)
        bv = (ti - xi) + occ
        xb = bv if bv > 0 else 0.0
        kb = i if (i < nle and xb == ti) else ssl(T, xb)
        kb = min(kb, n - 2)
        tb0, tb1, gb0, gb1 = T[kb], T[kb + 1], G[kb], G[kb + 1]
        da = (xa - st["ta0"]) / (st["ta1"] - st["ta0"])
        gi = st["ga0"] * (1.0 - da) + st["ga1"] * da
        if xb == tb0:
            go = gb0 * 1.0 + gb1 * 0.0
        else:
            db = (xb - tb0) / (tb1 - tb0)
            go = gb0 * (1.0 - db) + gb1 * db
        st["awin"] = gi if av >= 0 else 0.0
        st["awout"] = go if bv >= 0 else 0.0
        st["nev"] += 1
        return (st["awout"] - st["awin"]) + G0

    def upd(v):
        if v > st["mx"]:
            st["mx"] = v

    def hi_own(i):
        """the variant's bound of AW_OUT(b_i) for knot i alone: G[i] when b_i = t_i exactly"""
        k2 = min(i + koff, n - 1)
        if variant == 1 and i < nle and occ == xi:
            bv = (tau(i) - xi) + occ
            if bv == tau(i):
                return G[i], k2
        return G[k2], k2

    av = av_of(c)
    xa = av if av > 0 else 0.0
    seek(xa)
    upd(exact(c, av, xa))
    kc = st["ka"]
    ub_left = st["awout"]
    LA = st["awin"]
    i = c + 1
    while i < ntau:
        st["trips"] += 1
        av = av_of(i)
        xa = av if av > 0 else 0.0
        fwd(xa)
        lb = st["ga0"] if av >= 0 else 0.0
        LA = LA if LA > lb else lb
        V = (((st["mx"] - G0) + LA) - M) - dd
        hi, k2 = hi_own(i)
        if variant == 2:
            k2 = min(i + koff_of(i), n - 1)
            hi = G[k2]
        if hi > V:
            upd(exact(i, av, xa))
            LA = st["awin"]
            i += 1
            continue
        if variant == 1 and G[k2] > V:  # knot i pruned by its own bound only: step past it
            i += 1
            continue
        # skip every j with G[j + koff] <= V (gallop)
        kl = bisect.bisect_right(G, V, k2) - 1  # G nondecreasing here (mono columns)
        if kl >= n - 1:
            break
        inext = kl + 1 - koff_of(i)
        if variant == 2 and koff_of(i) == 0 and not (T[kl] <= 2.0 * xi):
            inext = max(kl + 1 - koff, i + 1)
        an = av_of(inext)
        seek(an if an > 0 else 0.0)
        i = inext
    UB = ub_left
    av = av_of(c)
    seek(av if av > 0 else 0.0)
    i = c - 1
    while i >= 0:
        st["trips"] += 1
        k2 = min(i + koff_of(i), n - 1)
        g2 = G[k2] if G[k2] > 0.0 else 0.0
        UB = UB if UB < g2 else g2
        Vp = (((UB + G0) + M) - st["mx"]) + dd
        if not (Vp - dd > 0.0):
            break
        av = av_of(i)
        xa = av if av > 0 else 0.0
        bwd(xa)
        lb = st["ga0"] if av >= 0 else 0.0
        Vi = Vp
        if variant == 1:
            h, _ = hi_own(i)
            h = h if h > 0.0 else 0.0
            ui = UB if UB < h else h
            Vi = (((ui + G0) + M) - st["mx"]) + dd
        if not (lb >= Vi):
            upd(exact(i, av, xa))
            UB = UB if UB < st["awout"] else st["awout"]
            i -= 1
            continue
        if not (lb >= Vp):  # pruned by knot i's own bound only
            i -= 1
            continue
        ks = first_ge_down(lambda k: G[k], st["ka"], Vp)
        tk = T[ks]
        j = first_ge_down(av_of, i, tk)
        if j == 0:
            break
        inext = j - 1
        an = av_of(inext)
        seek(an if an > 0 else 0.0)
        i = inext
    return st["mx"], st["nev"], st["trips"]


def main(ncol=16, ustride=8):
    g = sbr.fig5_grid(2048)
    cols = np.linspace(0, 2047, ncol).astype(int)
    tot = {0: 0, 1: 0, 2: 0}
    trips = {0: 0, 1: 0, 2: 0}
    npts = 0
    for ci in cols:
        beta = g.beta[ci]
        t, G, _ = O.learn_logistic(beta, 30.0)
        n = len(t)
        if np.any(np.diff(G) < 0):
            continue  # drawdown columns: dd > 0 (kept simple here)
        T, Gl = t.tolist(), G.tolist()
        nle = bisect.bisect_right(T, 15.0)
        ntau = nle if T[nle - 1] == 15.0 else nle + 1
        lo = bisect.bisect_right(Gl, 0.5) - 1
        thalf = T[lo] + (0.5 - Gl[lo]) * (T[lo + 1] - T[lo]) / (Gl[lo + 1] - Gl[lo])
        koff = 1 if all(T[i + 1] - T[i] > 1e-15 * T[-1] for i in range(n - 1)) else 2
        for uj in range(0, 2048, ustride):
            o = O.equilibrium_paths(t, G, beta, 15.0, 30.0, g.u[uj], 0.5, 0.6, 0.01)
            if not (o["status"] & sbr.STATUS["SBR_RUN"]):
                continue
            xi, tin, tout = o["xi"], o["tau_in_unc"], o["tau_out_unc"]
            icc = xi if tin >= xi else tin
            occ = xi if tout > xi else tout
            tstar = thalf + 0.5 * ((xi - icc) + (xi - occ))
            c = ssl(T, max(tstar, T[0]), 0, max(nle, 1) - 1)
            c = min(c, ntau - 1)
            for v in (0, 1, 2):
                mx, nev, tr = aw_scan(T, Gl, n, ntau, nle, 15.0, xi, icc, occ, Gl[0], 0.0, c, koff, v)
                assert mx == o["aw_max"], (ci, uj, v, mx, o["aw_max"])
                tot[v] += nev
                trips[v] += tr
            npts += 1
    print(f"{npts} run points: exact evaluations per point shipped {tot[0] / npts:.2f}, "
          f"own-knot bound {tot[1] / npts:.2f}, own-knot run bounds {tot[2] / npts:.2f}; loop trips "
          f"{trips[0] / npts:.2f} / {trips[1] / npts:.2f} / {trips[2] / npts:.2f}")


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
