"""Workgroup timeline of one config-3 equilibrium_kernel launch (diagnostic).

Needs a libsbr built with -DSBR_EQ_WGTIME (tools/build_variant.sh wgtime "-DSBR_EQ_WGTIME"),
selected with SBR_LIB.  Runs one 2048x2048 grid through the one-grid batch entry point,
reads every workgroup's start / end (100 MHz realtime clock) and hardware ids, and prints a
JSON summary: kernel span, concurrency profile (how many workgroups were resident over
time), per-column durations and the tail after the last workgroup started.
"""
import ctypes
import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))
import sbr  # noqa: E402
from sbr import _lib  # noqa: E402


def main():
    n = int(os.environ.get("WG_N", "2048"))
    flags = int(os.environ.get("WG_FLAGS", "0"), 0)
    dev = torch.device("cuda", 0)
    amt = sbr.julia_range("0.0001", "1", n)
    beta = torch.from_numpy(1.0 / amt).to(dev)[None, :]
    eta = torch.full((1, n), 15.0, dtype=torch.float64, device=dev)
    t_end = torch.full((1, n), 30.0, dtype=torch.float64, device=dev)
    u = torch.from_numpy(sbr.julia_range("0.001", "1", n)).to(dev)
    out = {k: torch.empty(1, n * n, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
    out["status"] = torch.empty(1, n * n, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(1, n * n, dtype=torch.int32, device=dev)
    eng = sbr.Engine(0)
    stream = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        eng.sweep_baseline_batch_dev(beta, eta, t_end, u, 0.5, 0.6, 0.01, 1e-4, out, stream=stream, flags=flags)
    torch.cuda.synchronize(dev)
    lib = ctypes.CDLL(str(_lib.LIB_PATH))
    nwg = n  # one workgroup per column at n_u <= 4096
    t2 = (ctypes.c_ulonglong * (2 * nwg))()
    hw2 = (ctypes.c_uint * (2 * nwg))()
    rc = lib.sbr_diag_wgtime_read(t2, hw2, nwg)
    assert rc == 0, rc
    t = np.frombuffer(t2, dtype=np.uint64).reshape(nwg, 2).astype(np.int64)
    hw = np.frombuffer(hw2, dtype=np.uint32).reshape(nwg, 2)
    t = (t - t[:, 0].min()) * 10.0 / 1000.0  # 100 MHz ticks -> microseconds
    start, end = t[:, 0], t[:, 1]
    dur = end - start
    span = float(end.max())
    grid = np.linspace(0, span, 401)
    conc = np.array([int(((start <= x) & (end > x)).sum()) for x in grid])
    status = out["status"][0].cpu().numpy().view(np.uint32).reshape(n, n)
    run = ((status & sbr.STATUS["SBR_RUN"]) > 0).sum(axis=1)
    xcc = hw[:, 1] & 0xF
    cu = (hw[:, 0] >> 8) & 0xF
    se = (hw[:, 0] >> 13) & 0x7
    order = np.argsort(end)[::-1]
    res = {
        "span_us": span,
        "last_start_us": float(start.max()),
        "tail_after_last_start_us": float(span - start.max()),
        "mean_concurrency": float(conc.mean()),
        "max_concurrency": int(conc.max()),
        "concurrency_deciles": [int(c) for c in conc[::40]],
        "frac_span_below_half_max": float((conc < conc.max() / 2).mean()),
        "dur_us": {"mean": float(dur.mean()), "median": float(np.median(dur)), "p90": float(np.percentile(dur, 90)),
                   "max": float(dur.max())},
        "dur_by_column_decile_us": [float(dur[i:i + n // 10].mean()) for i in range(0, n, n // 10)],
        "run_by_column_decile": [float(run[i:i + n // 10].mean()) for i in range(0, n, n // 10)],
        "corr_dur_run": float(np.corrcoef(dur, run)[0, 1]),
        "last10_columns": [{"col": int(c), "start": float(start[c]), "end": float(end[c]), "run": int(run[c])}
                           for c in order[:10]],
        "wg_per_xcc": np.bincount(xcc, minlength=8).tolist(),
        "busy_us_per_xcc": [float(dur[xcc == x].sum()) for x in range(8)],
        "distinct_cu": int(len(set(zip(xcc.tolist(), se.tolist(), cu.tolist())))),
    }
    print(json.dumps(res))
    outp = os.environ.get("WG_OUT")
    if outp:
        np.savez(outp, start=start, end=end, hw=hw, run=run)


if __name__ == "__main__":
    main()
