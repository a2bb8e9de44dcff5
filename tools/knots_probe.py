"""Latency breakdown of sbr_equilibrium_on_knots (the drop-in's per-u call): Python mirror,
Engine binding with / without paths, and a bare ctypes call on preallocated buffers; run it
under `rocprofv3 --kernel-trace --stats` for the kernel share.  Prints one JSON line."""
import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
import torch  # noqa: E402

import sbr  # noqa: E402
from sbr import _lib  # noqa: E402

torch.cuda.init()
eng = sbr.Engine(0)
m = sbr.ModelParameters.make(beta=1.0, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
lr = sbr.solve_learning(m.learning, eng)
t, G = lr.learning_cdf.knots, lr.learning_cdf.coefs
us = sbr.julia_range("0.001", "0.2", 5000)[:2700]
N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
res = {}


def timed(name, fn):
    for j in range(50):
        fn(float(us[j]))
    t0 = time.perf_counter()
    for j in range(N):
        fn(float(us[j % len(us)]))
    res[name] = (time.perf_counter() - t0) / N * 1e6


timed("mirror_us", lambda u: sbr.get_AW_functions(
    sbr.solve_equilibrium_baseline(lr, sbr.ModelParameters.modify(m, u=u).economic, eng)))
timed("engine_paths_us", lambda u: eng.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01))
timed("engine_nopaths_us", lambda u: eng.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, u, 0.5, 0.6, 0.01,
                                                               paths=False))
# bare ctypes call, buffers preallocated
L = _lib.load()
n = len(t)
cap = n + 1
out = np.empty(6)
pb = np.empty(5 * cap)
soa = _lib.ResultSoA(*[out.ctypes.data + 8 * k for k in range(5)], out.ctypes.data + 40, out.ctypes.data + 44)
opts = _lib.default_opts()
uu = np.zeros(1)
nt = ctypes.c_int64()
pp = [pb.ctypes.data + 8 * cap * k for k in range(5)]


def bare(u, paths):
    uu[0] = u
    return L.sbr_equilibrium_on_knots(eng._ctx, t.ctypes.data, G.ctypes.data, n, 1.0, 15.0, 30.0, uu.ctypes.data, 1,
                                      0.5, 0.6, 0.01, ctypes.byref(opts), ctypes.byref(soa),
                                      *(pp if paths else [None] * 5), cap, ctypes.byref(nt))


timed("bare_paths_us", lambda u: bare(u, True))
timed("bare_nopaths_us", lambda u: bare(u, False))
# a whole u vector in one call (the batched form of the same loop)
t0 = time.perf_counter()
for _ in range(20):
    eng.equilibrium_on_knots(t, G, 1.0, 15.0, 30.0, us, 0.5, 0.6, 0.01, paths=False)
res["vector_2700_us_per_point"] = (time.perf_counter() - t0) / 20 / len(us) * 1e6
res["n_knots"] = n
res["calls"] = N
print(json.dumps(res), flush=True)
