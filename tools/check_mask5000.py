#!/usr/bin/env python3
"""CPU check of the 5000² paper run mask at each column's boundary only: for
column c with paper prefix P (tests/golden/fig5_prefix.json), u index P-1 must
be a run and P must not.  Uses the oracle (test infrastructure), ~1 min."""
import json
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / "oracle"), str(REPO / "replication-social-bank-runs_amd")]
import oracle as O  # noqa: E402
import sbr  # noqa: E402

grid = sbr.fig5_grid(5000)
pref = np.array(json.loads((REPO / "tests/golden/fig5_prefix.json").read_text())["n5000"]["prefix"])
RUN = sbr.STATUS["SBR_RUN"]


def col(c):
    P = int(pref[c])
    idx = [i for i in (P - 1, P) if 0 <= i < len(grid.u)]
    r = O.sweep_baseline([grid.beta[c]], 15.0, 30.0, grid.u[idx], grid.p, grid.kappa, grid.lam, grid.x0)
    run = (r["status"][0] & RUN) > 0
    ok = all(run[k] == (i < P) for k, i in enumerate(idx))
    return c, ok


bad = []
with ThreadPoolExecutor(8) as ex:
    for c, ok in ex.map(col, range(len(grid.beta))):
        if not ok:
            bad.append(c)
print(json.dumps({"bad_columns": bad}))
