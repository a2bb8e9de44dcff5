"""Per-phase shader cycles of single social points run alone (SBR_FLAG_DIAG_SOCIAL_PROF),
first `max_iter` fixed-point iterates; for A/B of libsbr builds (SBR_LIB=...).
usage: python tools/social_phase_probe.py [max_iter]   (JSON lines on stdout)"""
import json
import sys

import torch

sys.path.insert(0, "replication-social-bank-runs_amd")
import sbr  # noqa: E402

mi = int(sys.argv[1]) if len(sys.argv) > 1 else 8
dev = torch.device("cuda", 0)
eng = sbr.Engine(0)
names = ("cmp_prelude", "ode", "hazard_scan", "bisection", "aw_norm", "damping_awmax")
for beta, u in ((100.0, 0.001), (0.5069092424137213, 0.36071819960861057)):
    eta = 30.0 / 0.9
    b = torch.tensor([beta], dtype=torch.float64, device=dev)
    e = torch.tensor([eta], dtype=torch.float64, device=dev)
    uu = torch.tensor([u], dtype=torch.float64, device=dev)
    cmp = torch.from_numpy(sbr.julia_range(0.0, eta, 1000)).to(dev)[None, :]
    out = {k: torch.empty(1, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
    out["status"] = torch.empty(1, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(1, dtype=torch.int32, device=dev)
    out["fp_iters"] = torch.empty(1, dtype=torch.int32, device=dev)
    out["rk_steps"] = torch.empty(1, dtype=torch.int64, device=dev)
    eng.social_prof_read()
    s = torch.cuda.current_stream(dev).cuda_stream
    eng.sweep_social_dev(b, e, uu, 0.99, 0.25, 0.25, cmp, 1e-4, out, max_iter=mi, stream=s,
                         flags=sbr._lib.SBR_FLAG_DIAG_SOCIAL_PROF)
    torch.cuda.synchronize(dev)
    pr = eng.social_prof_read()
    tot = max(sum(pr[:6]), 1)
    print(json.dumps(dict(beta=beta, u=u, max_iter=mi, rk_steps=int(out["rk_steps"][0]),
                          cycles_total=tot, share={k: pr[i] / tot for i, k in enumerate(names)},
                          cycles_per_rk_step_ode=pr[1] / max(pr[7], 1),
                          cycles_per_rk_step_all=tot / max(pr[7], 1))), flush=True)
