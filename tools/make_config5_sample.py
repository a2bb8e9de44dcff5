#!/usr/bin/env python3
"""Golden fixture for the config-5 GPU parity test (tests/test_gpu_social.py): the CPU
oracle (test infrastructure; oracle/sbr_oracle.c social_point, a restatement of
solve_equilibrium_social_learning, social_learning_solver.jl:63-263) on an 8 β × 4 u
sample of BASELINE config 5 (β = 1/range(0.01, 2, 512), u = range(0.001, 1, 512),
m_social's p = 0.99, κ = λ = 0.25, η = 30/0.9 carried, tol = 1e-4, max_iter = 500),
including the fringe corner β = 100, u = 0.001.  Writes tests/golden/config5_sample.npz.

With --stride S: every S-th β × every S-th u of the 512² axes (S = 16: a stratified
1,024-point sample, corner included) → tests/golden/config5_sample_<n>.npz."""
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO), str(REPO / "replication-social-bank-runs_amd")]
import oracle.oracle as O  # noqa: E402
import sbr  # noqa: E402

BI = np.array([0, 73, 146, 219, 292, 365, 438, 511])
UI = np.array([0, 3, 170, 511])
ETA = 30.0 / 0.9


def main():
    bi, ui, name = BI, UI, "config5_sample.npz"
    if "--stride" in sys.argv:
        s = int(sys.argv[sys.argv.index("--stride") + 1])
        bi = ui = np.arange(0, 512, s)
        name = f"config5_sample_{len(bi) * len(ui)}.npz"
    beta = (1.0 / sbr.julia_range("0.01", "2", 512))[bi]
    u = sbr.julia_range("0.001", "1", 512)[ui]
    cmp = np.stack([sbr.julia_range(0.0, ETA, 1000)] * len(beta))
    t0 = time.time()
    o = O.sweep_social(beta, ETA, u, 0.99, 0.25, 0.25, cmp, tol=1e-4, max_iter=500, nthreads=8, stats=True)
    dt = time.time() - t0
    keep = {k: o[k] for k in ("xi", "tau_in_unc", "tau_out_unc", "aw_max", "tol", "status", "iters", "fp_iters")}
    np.savez_compressed(REPO / "tests" / "golden" / name, beta_idx=bi, u_idx=ui, beta=beta, u=u, **keep)
    print(f"{len(beta)}x{len(u)} points in {dt:.1f} s; fp_iters max {int(o['fp_iters'].max())}; "
          f"status {sorted(set(int(s) for s in o['status'].ravel()))}")
    if "stats" in o:
        print("max knots / acc / rej per point:", o["stats"][..., 0].max(), o["stats"][..., 1].max(), o["stats"][..., 2].max())


if __name__ == "__main__":
    main()
