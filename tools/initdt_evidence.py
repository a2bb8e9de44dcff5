"""Which exponent does the reference's initial-dt heuristic use?  Evidence from every
reference figure that can tell.

ode_determine_initdt computes dt₁ = (0.01 / max(d₁, d₂))^(1/(order+1)).  The restatement
takes Tsit5's order 5 (exponent 1/6); the alternative reading is 1/5.  The first dt moves
every knot of the adaptive grid, so the choice shows up in the figures' exact boundaries.
This script runs the CPU oracle with each exponent on:
  * Fig 4 (scripts/1_baseline.jl:137-192): the run/no-run boundary of the 5000-point u sweep
    (the figure has exactly 2718 leading runs) and the AW_max / ξ curves;
  * Fig 5 at 500² (1_baseline.jl:210-267): the run mask, cell for cell (87,554 run cells);
  * Fig 5 at 5000² (comp_stat_cross_heatmap_AW_large.pdf): every column's boundary pair
    (u index P−1 runs, P does not);
  * Fig 3 main: ξ against the figure's 10.2155.
and the one cell any variant disagrees on under ±4-ulp perturbations of the first dt, and
writes the mismatch counts to profiles/r03_initdt_exponent.json.
Run: python tools/initdt_evidence.py   (≈ 2-4 minutes on 8 cores)"""
from __future__ import annotations

import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
sys.path.insert(0, str(REPO / "oracle"))
import oracle as O  # noqa: E402
import sbr  # noqa: E402

GOLD = REPO / "tests" / "golden"
RUN = sbr.STATUS["SBR_RUN"]


def evidence(form: int, den: int) -> dict:
    O.set_initdt(form, den)
    out = {"exponent": f"1/{den}", "form": ["(0.01/max_d)^(1/order)", "10^(-(2 + log10(max_d))/order)"][form]}
    # Fig 3 main
    t, G, _ = O.learn_logistic(1.0, 30.0)
    r = O.equilibrium(t, G, 1.0, 15.0, 30.0, 0.1, 0.5, 0.6, 0.01)
    g3 = json.loads((GOLD / "fig3_equilibria.json").read_text())["main"]
    out["fig3_main"] = {"xi": r["xi"], "figure_xi": g3["xi"], "abs_diff": abs(r["xi"] - g3["xi"]),
                        "knots": int(len(t))}
    # Fig 4
    g4 = json.loads((GOLD / "fig4_u_sweep.json").read_text())
    grid = sbr.fig4_grid(5000)
    r = O.apply_early_exit(O.sweep_baseline(grid.beta, grid.eta, grid.t_end, grid.u, 0.5, 0.6, 0.01), 5)
    run = (r["status"][0] & RUN) > 0
    n_lead = int(np.argmin(run)) if not run.all() else len(run)
    n = g4["n_run_prefix"]
    out["fig4"] = {"leading_runs": n_lead, "figure_leading_runs": n, "run_cells": int(run.sum()),
                   "aw_max_max_abs_dev": float(np.max(np.abs(r["aw_max"][0, :n] - np.array(g4["aw_max"])))),
                   "xi_max_abs_dev": float(np.max(np.abs(r["xi"][0, :n] - np.array(g4["xi"]))))}
    # Fig 5 500²
    pref5 = json.loads((GOLD / "fig5_prefix.json").read_text())
    grid = sbr.fig5_grid(500)
    r = O.apply_early_exit(O.sweep_baseline(grid.beta, grid.eta, grid.t_end, grid.u, 0.5, 0.6, 0.01), 5)
    run = (r["status"] & RUN) > 0
    mask = np.zeros_like(run)
    for c, k in enumerate(pref5["n500"]["prefix"]):
        mask[c, :k] = True
    diff = np.argwhere(run != mask)
    out["fig5_500"] = {"run_cells": int(run.sum()), "figure_run_cells": int(mask.sum()),
                       "mismatched_cells": int(len(diff)),
                       "mismatches": [{"beta": float(grid.beta[c]), "u": float(grid.u[j]), "engine_run": bool(run[c, j])}
                                      for c, j in diff[:10]]}
    # Fig 5 5000² boundary pairs
    grid = sbr.fig5_grid(5000)
    pref = np.array(pref5["n5000"]["prefix"])

    def col(c):
        P = int(pref[c])
        idx = [i for i in (P - 1, P) if 0 <= i < len(grid.u)]
        rr = O.sweep_baseline([grid.beta[c]], 15.0, 30.0, grid.u[idx], grid.p, grid.kappa, grid.lam, grid.x0)
        ok = (rr["status"][0] & RUN) > 0
        return all(ok[k] == (i < P) for k, i in enumerate(idx))

    with ThreadPoolExecutor(8) as ex:
        ok = list(ex.map(col, range(len(grid.beta))))
    bad = [c for c, v in enumerate(ok) if not v]
    out["fig5_5000_boundaries"] = {"columns": len(ok), "mismatched_columns": len(bad), "first": bad[:10]}
    return out


def knife_edge(forms=((0, 6), (0, 5), (1, 5), (1, 6)), ulps=range(-4, 5)) -> dict:
    """The one Fig 5 cell any variant disagrees on — (β₂₈₄, u₉₅), no run in the figure —
    with the first dt moved by -4 … +4 ulps: how robust is each variant's verdict there?"""
    g = sbr.fig5_grid(500)
    c, j = 284, 95
    out = {"cell": {"beta": float(g.beta[c]), "u": float(g.u[j]), "figure": "no run"}, "variants": []}
    for form, den in forms:
        runs = []
        for k in ulps:
            O.set_initdt(form, den)
            O.set_initdt_ulps(k)
            r = O.sweep_baseline([g.beta[c]], 15.0, 30.0, g.u[j:j + 1], 0.5, 0.6, 0.01)
            runs.append(bool(r["status"][0, 0] & RUN))
        out["variants"].append({"form": ["(0.01/max_d)^(1/order)", "10^(-(2 + log10(max_d))/order)"][form],
                                "exponent": f"1/{den}", "ulps": list(ulps), "run": runs,
                                "agrees_with_figure": f"{sum(not x for x in runs)}/{len(runs)}"})
    O.set_initdt_ulps(0)
    O.set_initdt(0, 6)
    return out


def main():
    O.build()
    t0 = time.time()
    res = {"what": "initial-dt exponent of ode_determine_initdt: 1/6 (Tsit5 order 5 + 1) vs 1/5; mismatch counts "
                   "against the reference's committed figures (tools/initdt_evidence.py)",
           "runs": [evidence(0, 6), evidence(0, 5), evidence(1, 5), evidence(1, 6)]}
    res["knife_edge_cell"] = knife_edge()
    O.set_initdt(0, 6)
    res["seconds"] = round(time.time() - t0, 1)
    out = REPO / "profiles" / "r03_initdt_exponent.json"
    out.write_text(json.dumps(res, indent=1) + "\n")
    for r in res["runs"]:
        print(r["form"], r["exponent"], "fig4 leading", r["fig4"]["leading_runs"], "500² mismatched", r["fig5_500"]["mismatched_cells"],
              "5000² mismatched columns", r["fig5_5000_boundaries"]["mismatched_columns"], "fig3 dxi",
              r["fig3_main"]["abs_diff"])
    for v in res["knife_edge_cell"]["variants"]:
        print("cell (β284, u95):", v["form"], v["exponent"], "agrees with the figure for", v["agrees_with_figure"],
              "of the ±4-ulp first steps")


if __name__ == "__main__":
    main()
