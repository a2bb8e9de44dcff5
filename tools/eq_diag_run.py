"""One config-3 grid through the one-grid batch entry point with a diagnostic flag
(for per-phase PMC passes: rocprofv3 --pmc ... -- python3 tools/eq_diag_run.py FLAG).
FLAG: 0 full, 0x100 stop after the crossing scan, 0x200 stop after the bisection."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
import sbr  # noqa: E402

flags = int(sys.argv[1], 0) if len(sys.argv) > 1 else 0
n = 2048
dev = torch.device("cuda", 0)
beta = torch.from_numpy(1.0 / sbr.julia_range("0.0001", "1", n)).to(dev)[None, :]
eta = torch.full((1, n), 15.0, dtype=torch.float64, device=dev)
t_end = torch.full((1, n), 30.0, dtype=torch.float64, device=dev)
u = torch.from_numpy(sbr.julia_range("0.001", "1", n)).to(dev)
out = {k: torch.empty(1, n * n, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
out["status"] = torch.empty(1, n * n, dtype=torch.int32, device=dev)
out["iters"] = torch.empty(1, n * n, dtype=torch.int32, device=dev)
eng = sbr.Engine(0)
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(3):
    eng.sweep_baseline_batch_dev(beta, eta, t_end, u, 0.5, 0.6, 0.01, 1e-4, out, stream=s, flags=flags)
torch.cuda.synchronize(dev)
print("ok", flags)
