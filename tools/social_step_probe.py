"""µs per RK step of single social points run alone (first `max_iter` fixed-point
iterates), for A/B of libsbr builds (SBR_LIB=...).
usage: python tools/social_step_probe.py [max_iter]   (JSON lines on stdout)"""
import json
import sys
import time

import torch

sys.path.insert(0, "replication-social-bank-runs_amd")
torch.cuda.init()
import sbr  # noqa: E402

mi = int(sys.argv[1]) if len(sys.argv) > 1 else 8
eng = sbr.Engine(0)
for beta, u in ((100.0, 0.001), (0.5069092424137213, 0.36071819960861057)):
    eng.sweep_social([beta], 30.0 / 0.9, [u], 0.99, 0.25, 0.25, max_iter=1)  # warm
    eng.timing_enable(True)
    t0 = time.time()
    r = eng.sweep_social([beta], 30.0 / 0.9, [u], 0.99, 0.25, 0.25, max_iter=mi)
    wall = time.time() - t0
    lm, em, n = eng.timing_read()
    eng.timing_enable(False)
    steps = int(r["rk_steps"][0, 0])
    print(json.dumps(dict(beta=beta, u=u, max_iter=mi, wall_s=wall, iter_ms=em, rk_steps=steps,
                          fp_iters=int(r["fp_iters"][0, 0]), us_per_step=em * 1e3 / max(steps, 1))), flush=True)
