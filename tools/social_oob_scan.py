#!/usr/bin/env python3
"""Scan small-u points of BASELINE config 5 on the CPU oracle (test infrastructure) for fixed
points that end in the reference's BoundsError (SBR_OOB, with or without SBR_ODE_FAILED);
the GPU tests use the cheap ones.  Prints (β index, u index, status, fp_iters, seconds)."""
import sys, time, numpy as np, multiprocessing as mp
REPO = __import__("pathlib").Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO)); sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
ETA = 30.0/0.9
def run(args):
    bi, ui = args
    import oracle.oracle as O, sbr
    beta = 1.0 / sbr.julia_range("0.01", "2", 512); u = sbr.julia_range("0.001", "1", 512)
    cmp = sbr.julia_range(0.0, ETA, 1000)
    t0 = time.time()
    o = O.sweep_social([beta[bi]], ETA, [u[ui]], 0.99, 0.25, 0.25, cmp, tol=1e-4, max_iter=500)
    return bi, ui, int(o["status"][0,0]), int(o["fp_iters"][0,0]), time.time()-t0
if __name__ == "__main__":
    import sbr
    cands = [(b, uu) for b in (0, 5, 10, 20, 40, 60, 100) for uu in (0, 1, 2, 3, 4, 6)]
    with mp.Pool(8) as p:
        res = []
        for r in p.imap_unordered(run, cands):
            print(r, "OOB" if r[2] & 0x80 else "", "FAILED" if r[2] & 0x4000 else "", flush=True)
