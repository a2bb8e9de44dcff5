"""Debug: bench-style pipelined hetero batch vs single sweep on one config-4 shard (GPU)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "replication-social-bank-runs_amd")
import sbr

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
g = sbr.hetero_config4(n, n, K=8)
K, nb, nu = g.K, g.betas.shape[0], len(g.u)
T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
eng = sbr.Engine(0)
stream = torch.cuda.current_stream(dev).cuda_stream
ref = eng.sweep_hetero(g.betas, g.dist, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, with_groups=False)
for nbat in (1, 2, 3):
    out = {k: torch.empty(nbat, nb * nu, dtype=torch.float64, device=dev) for k in ("xi", "aw_max", "tol")}
    out["status"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    betas = T(g.betas).unsqueeze(0).repeat(nbat, 1, 1).contiguous()
    eta = T(g.eta).unsqueeze(0).repeat(nbat, 1).contiguous()
    t_end = T(g.t_end).unsqueeze(0).repeat(nbat, 1).contiguous()
    eng.sweep_hetero_batch_dev(K, betas, T(g.dist), eta, t_end, T(g.u), g.p, g.kappa, g.lam, g.x0, out, stream=stream)
    torch.cuda.synchronize(dev)
    for k in range(nbat):
        st = out["status"][k].cpu().numpy().view(np.uint32)
        aw = out["aw_max"][k].cpu().numpy()
        print(nbat, k, "status_eq", np.array_equal(st, ref["status"].ravel()),
              "aw_eq", np.array_equal(aw, ref["aw_max"].ravel(), equal_nan=True),
              "run", float(((st & sbr.STATUS["SBR_RUN"]) > 0).mean()), flush=True)
print("ref run", float(((ref["status"] & sbr.STATUS["SBR_RUN"]) > 0).mean()))
