"""Diagnose Fig 5 5000² mask differences: default vs exhaustive vs oracle on the differing columns."""
import json, sys
from pathlib import Path
import numpy as np
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd")); sys.path.insert(0, str(REPO / "oracle"))
import sbr, oracle as O
eng = sbr.Engine(0)
grid = sbr.fig5_grid(5000)
pref = np.array(json.loads((REPO / "tests/golden/fig5_prefix.json").read_text())["n5000"]["prefix"])
a = eng.sweep_baseline(grid, early_exit=5, with_iters=False)
b = eng.sweep_baseline(grid, early_exit=5, with_iters=False, exhaustive=True)
ra = (a["status"] & 1) > 0
rb = (b["status"] & 1) > 0
ga = np.array([np.argmin(r) if not r.all() else len(r) for r in ra])
gb = np.array([np.argmin(r) if not r.all() else len(r) for r in rb])
print("default vs golden cols differ:", np.nonzero(ga != pref)[0][:10], "exhaustive vs golden:", np.nonzero(gb != pref)[0][:10])
print("default vs exhaustive status differ:", int((a["status"] != b["status"]).sum()))
for c in sorted(set(np.nonzero(ga != pref)[0][:5]) | set(np.nonzero(gb != pref)[0][:5])):
    print("col", c, "beta", repr(grid.beta[c]), "golden prefix", pref[c], "default", ga[c], "exhaustive", gb[c])
    sub = grid.subset([c])
    o = O.apply_early_exit(O.sweep_baseline(sub.beta, sub.eta, sub.t_end, sub.u, 0.5, 0.6, 0.01), 5)
    ro = (o["status"][0] & 1) > 0
    go = np.argmin(ro) if not ro.all() else len(ro)
    print("   oracle prefix", go)
    k = min(pref[c], ga[c]) - 1
    for j in range(max(0, k - 2), min(5000, k + 4)):
        print("   j", j, "u", repr(grid.u[j]), "gpu", hex(a["status"][c, j]), a["xi"][c, j], "orc", hex(o["status"][0, j]), o["xi"][0, j])
