"""Time the slowest config-5 social points alone (default knot capacity with
overflow restarts vs one large capacity), with per-pass kernel time.
usage: python tools/social_tail_probe.py [beta2]   (writes JSON lines to stdout)"""
import json
import sys
import time

import torch

sys.path.insert(0, "replication-social-bank-runs_amd")
torch.cuda.init()
import sbr  # noqa: E402

eng = sbr.Engine(0)
eng.timing_enable(True)
runs = [(100.0, 0.001, 0), (100.0, 0.001, 1 << 21)]
if len(sys.argv) > 1:
    runs.append((float(sys.argv[1]), 0.001, 0))
for beta, u, cap in runs:
    t0 = time.time()
    r = eng.sweep_social([beta], 30.0 / 0.9, [u], 0.99, 0.25, 0.25, max_iter=500, knot_capacity=cap)
    wall = time.time() - t0
    lm, em, n = eng.timing_read()
    rec = dict(beta=beta, u=u, cap=cap, wall_s=wall, passes=n, iter_ms=em, init_ms=lm,
               rk_steps=int(r["rk_steps"][0, 0]), fp_iters=int(r["fp_iters"][0, 0]),
               status=hex(int(r["status"][0, 0])), xi=float(r["xi"][0, 0]))
    rec["us_per_step"] = em * 1e3 / max(rec["rk_steps"], 1)
    print(json.dumps(rec), flush=True)
