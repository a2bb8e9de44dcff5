#!/usr/bin/env python3
"""Benchmark: equilibria solved per second on the β×u grid (FP64), BASELINE.json's metric.

Workload (BASELINE config 3): the Fig 5 grid of scripts/1_baseline.jl:210-212 at
2048×2048 — ave_meeting_time = range(1e-4, 1, 2048), β = 1/amt, u = range(0.001, 1,
2048), η = 15 and tspan = (0, 30) for every β (copy-modify carry-over) — 4,194,304
equilibria per GPU.  One step = one full sweep: learning (Tsit5 + hazard) for every
β column, then buffers + ξ bisection + AW_max for every (β, u), every point solved
(no early exit), inputs already resident in HBM, results written to HBM.  The K
timed steps are K grids handed to ONE sbr_sweep_baseline_batch_dev call: the
learning stage (latency-bound, one serial ODE per β lane, 32 waves per grid) of up
to 24 grids runs as one launch of one wave per SIMD, then the equilibria run back
to back with nothing beside them (a longer batch learns its next group beside
them).  Every step's learning and equilibrium run in full inside the timed region
(--no-pipeline: one serial sweep call per step); the learning launch (≈3 ms, the
slowest column's serial chain) is the fill the K steps share.  The batch's HBM
workspace is allocated before the warmup (sbr_batch_reserve), outside the timed
region, like the result tensors.

N GPUs (torchrun, one process per GPU, RCCL): weak scaling — rank r owns the β
columns r, r+N, r+2N, … of a 2048·N-column grid (same u axis), so per-GPU work is
fixed.  Every step's full result SoA (ξ, τ̄_IN, τ̄_OUT, AW_max, tol, status, bisection
iterations: 48 B per point) is collected over RCCL/xGMI: step k's grid on rank k mod N,
N consecutive steps by one all-to-all per field (sbr.distributed.StepCollector: every
link carries a share in both directions; a gather of every step to rank 0 would be
capped by rank 0's inbound links), issued on its own stream once those steps' results
exist (sbr_batch_wait) so that it overlaps the later steps' sweeps.  value = all ranks'
equilibria × steps / max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "replication-social-bank-runs_amd"))


# ---- N-rank launcher: `python bench.py --gpus N` without a launcher's WORLD_SIZE starts N rank
# processes itself (one per GPU, as torchrun would), before this process imports torch or libsbr:
# the parent never initialises HIP; it waits for its children and exits with their status ----
def launch_plan(argv: list[str], env: dict, port: int) -> list[tuple[list[str], dict]]:
    """(command, environment) of every rank process for `python bench.py argv`, or [] when this
    process is itself a rank (a launcher set WORLD_SIZE) or --gpus is 1."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--gpus", type=int, default=1)
    n = pre.parse_known_args(argv)[0].gpus
    if "WORLD_SIZE" in env or n <= 1:
        return []
    plan = []
    for r in range(n):
        e = dict(env)
        e.update(WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plan.append(([sys.executable, "-u", str(Path(__file__).resolve())] + list(argv), e))
    return plan


def world_of(gpus: int, env=None) -> tuple[int, int, int]:
    """(world, rank, local rank) of this process; a launcher's WORLD_SIZE must equal --gpus."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}: refusing a mismatched world")
    return world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(argv: list[str]) -> int | None:
    import signal
    import subprocess
    plan = launch_plan(argv, dict(os.environ), _free_port())
    if not plan:
        return None
    procs = [subprocess.Popen(cmd, env=e) for cmd, e in plan]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0 and rc == 0:
                    rc = r if r > 0 else 128 - r
                    for q in pending:  # one rank failed: the others would wait in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


if __name__ == "__main__":
    _rc = _launch(sys.argv[1:])
    if _rc is not None:
        sys.exit(_rc)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import sbr  # noqa: E402
from sbr import distributed as D  # noqa: E402

FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec (256 CU x 128 FLOP/clk x 2.4 GHz)

# Algorithmic flops per unit of work, SURVEY.md §8(d)'s counting convention (FMA = 2,
# add/sub/mul/div/exp/pow = 1, compares/branches/searches = 0), counted on the work the
# reference's algorithm defines — not on what the kernels execute (branch and bound
# evaluates far fewer AW knots; the executed FP64 work comes from the PMC counters).
F8_BUFFER = 12        # per point: optimal_buffer's two crossing interpolations (solver.jl:237,250)
F8_BISECT_ITER = 20   # per compute_ξ iteration: 4 lerps x 4 + 4 (solver.jl:326-372)
F8_AW_KNOT = 12       # per τ̄ knot of a run point's AW path: 2 lerps x 4 + 4 (solver.jl:511-524, 565)
F8_RK_STEP = 96       # per attempted Tsit5 step of a scalar ODE (94 + 2)
F8_HZ_KNOT = 15       # per τ̄ knot of hazard_rate (solver.jl:168-182)
PMC_SUMMARY = REPO / "profiles" / "pmc_latest.json"


def lib_sha() -> str:
    import hashlib
    return hashlib.sha256(sbr._lib.LIB_PATH.read_bytes()).hexdigest()[:16]


def pmc_of(kernel_prefix: str, workload: str):
    """(executed FP64 flops, HBM bytes) per launch of a kernel from the committed PMC summary
    (tools/pmc_summary.py -> profiles/pmc_latest.json), only when the counters were collected
    on this kernel's machine code (sbr.provenance.kernel_code_sha over libsbr.so) and
    workload; (None, None) otherwise.  Executed flops: 64·(ADD + MUL + TRANS) + 128·FMA over
    SQ_INSTS_VALU_*_F64 (wave instructions, every lane counted as active: an upper bound).
    Bytes: FETCH_SIZE×2 (gfx950) + WRITE_SIZE, MI355X_MICROARCH.md's correction."""
    from sbr import provenance
    try:
        pm = json.loads(PMC_SUMMARY.read_text())["workloads"][workload]["kernels"]
    except Exception:
        return None, None
    for k, c in pm.items():
        if not k.startswith(kernel_prefix):
            continue
        if c.get("code_sha16") is None or c["code_sha16"] != provenance.kernel_code_sha(k):
            return None, None
        ex = None
        if "SQ_INSTS_VALU_FMA_F64" in c:
            ex = (64 * (c.get("SQ_INSTS_VALU_ADD_F64", 0) + c.get("SQ_INSTS_VALU_MUL_F64", 0)
                        + c.get("SQ_INSTS_VALU_TRANS_F64", 0)) + 128 * c["SQ_INSTS_VALU_FMA_F64"])
        return ex, c.get("hbm_bytes_per_launch")
    return None, None


def pmc_social(rk_steps: float):
    """(executed FP64 flops, HBM bytes) of social_iter_kernel over a whole share, from the PMC run
    that tools/pmc_social.py folded into profiles/pmc_latest.json per attempted RK step (the first
    16 iterates of the config-5 share, where the bulk runs), scaled by this run's RK steps; only
    when the counters were taken on this kernel's machine code.  Bytes: FETCH_SIZE×2 + WRITE_SIZE."""
    from sbr import provenance
    try:
        c = json.loads(PMC_SUMMARY.read_text())["workloads"]["social_64x512_bulk16"]["kernels"]["social_iter_kernel"]
    except Exception:
        return None, None
    if c.get("code_sha16") is None or c["code_sha16"] != provenance.kernel_code_sha("social_iter_kernel"):
        return None, None
    ex = c.get("fp64_flops_executed_per_rk_step")
    by = c.get("hbm_bytes_per_rk_step")
    return (ex * rk_steps if ex is not None else None), (by * rk_steps if by is not None else None)


def roofline(kernel: str, flops: float, secs: float, pmc=(None, None), limiter="latency") -> dict:
    """roofline block for `kernel`: algorithmic flops per launch / average launch time.
    The roof the metric is priced against is the FP64 vector peak (no dense
    contraction: no MFMA; ≈10⁴ flop/B: not HBM); `bound` names what limits the kernel
    in practice (PMC: dependent search / division chains, wait and issue stalls)."""
    ach = flops / secs / 1e12 if secs > 0 else 0.0
    executed, traffic = pmc
    r = {"bound": limiter, "roof": "valu_fp64", "kernel": kernel, "achieved": ach, "peak": FP64_VALU_PEAK_TFLOPS,
         "unit": "TFLOP/s", "frac": ach / FP64_VALU_PEAK_TFLOPS, "traffic": traffic,
         "flops_per_launch": flops, "flop_convention": "SURVEY.md §8(d)"}
    if executed is not None and secs > 0:
        r["frac_executed"] = executed / secs / 1e12 / FP64_VALU_PEAK_TFLOPS
        r["executed_flops_per_launch"] = executed
    else:
        r["frac_executed"] = None
    return r


def usable_cores() -> int:
    """CPUs this process may use: the affinity set, capped by a cgroup v2 cpu.max quota."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            n = max(1, min(n, int(int(q) // int(per))))
    except Exception:
        pass
    return n


def host_info() -> dict:
    model = "unknown"
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {"nproc": os.cpu_count(), "usable": usable_cores(), "model": model}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=2048, help="β columns per GPU and u rows")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: the --n x --n grid (config 3) dealt over the N ranks (default: weak, "
                         "--n columns per rank)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="one-GPU rehearsal of a strong run: solve the β-column shard that rank --shard-rank of "
                         "a --shard-of-rank run owns")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one sbr_sweep_baseline_dev call per step (no learning/equilibrium overlap across steps)")
    ap.add_argument("--ready", action="store_true",
                    help="--no-pipeline: the per-column readiness schedule (SBR_FLAG_READY_SWEEP) instead of chunks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-verify", action="store_true",
                    help="skip checking the last timed grid against the oracle (12 sampled columns)")
    ap.add_argument("--cpu-stride", type=int, default=2, help="cpu_baseline samples every k-th β column")
    ap.add_argument("--phases", action="store_true",
                    help="also time the equilibrium kernel stopped after each stage (diagnostic flags)")
    ap.add_argument("--workload", choices=("baseline", "social", "hetero", "interest", "config1", "config2",
                                           "dropin", "launchcheck", "multihost"),
                    default="baseline",
                    help="baseline: BASELINE config 3 (the metric); social: config 5 per-GPU share; "
                         "hetero: config 4 (K = 8, 1024x1024 per GPU); interest: the interest-rate "
                         "extension on the Fig 5 grid (500x500 per GPU, r = 0.06, delta = 0.1); config1: "
                         "one Fig 3 equilibrium per call (latency); config2: one 500x500 Fig 5 sweep per "
                         "call with the 5-NaN early exit, host arrays in and out; dropin: the unchanged "
                         "scripts' per-u loops (Fig 4, Fig 5) through the drop-in, latency per call")
    ap.add_argument("--interest-n", type=int, default=500, help="interest: β columns per GPU and u rows")
    ap.add_argument("--hetero-n", type=int, default=1024, help="hetero: columns per GPU and u rows")
    ap.add_argument("--social-cols", type=int, default=64, help="social: β columns per GPU (config 5: 512/8)")
    ap.add_argument("--social-max-iter", type=int, default=500)
    ap.add_argument("--social-prof", action="store_true", help="social: per-phase cycle breakdown (diagnostic)")
    ap.add_argument("--social-dump", default="", help="social: save per-point status/fp_iters/rk_steps (.npz)")
    return ap.parse_args()


def main_small(a):
    """BASELINE configs 1 and 2, timed the way a drop-in caller pays them (host arrays in and
    out, one synchronous C-ABI call each; N = 1 only).
    config1: the Fig 3 main equilibrium (scripts/1_baseline.jl:82-86) — solve_learning +
    solve_equilibrium_baseline + get_AW as sbr_solve_point_paths (learning, hazard, buffers,
    ξ, the AW_cum path) — latency per call.
    config2: the Fig 5 500×500 grid (scripts/1_baseline.jl:210-267) — one sbr_sweep_baseline
    call with early_exit_nan_run = 5 — equilibria per second over the whole grid."""
    if world_of(a.gpus)[0] != 1:
        raise SystemExit(f"bench.py: --workload {a.workload} is a one-GPU latency line (--gpus 1)")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.init()
    eng = sbr.Engine(0)
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure: cpu_baseline leg only)
    if a.workload == "dropin":
        return main_dropin(a, eng, O)
    if a.workload == "multihost":
        return main_multihost(a)
    if a.workload == "config1":
        args = dict(beta=1.0, eta=15.0, t_end=30.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
        for _ in range(max(a.warmup, 1)):
            r = eng.solve_point_paths(**args)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            r = eng.solve_point_paths(**args)
        dt = (time.perf_counter() - t0) / a.steps
        res = {"metric": "single baseline equilibrium latency (Fig 3 main, host API)", "value": dt * 1e3,
               "unit": "ms per equilibrium", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": dt * 1e3, "higher_is_better": False, "scaling": None, "vs_baseline": None,
               "dtype": "f64", "data": "the reference's Fig 3 parameters",
               "config": {"workload": "config1: sbr_solve_point_paths(beta=1, eta=15, tspan=(0,30), u=0.1, "
                                      "p=0.5, kappa=0.6, lambda=0.01) (BASELINE config 1)"},
               "xi": r["xi"], "paper_cpu_seconds": 0.5, "libsbr_sha16": lib_sha()}
        if not a.no_cpu_baseline:
            O.build()
            n = 20
            t1 = time.perf_counter()
            for _ in range(n):
                t, G, _ = O.learn_logistic(1.0, 30.0)
                o = O.equilibrium(t, G, 1.0, 15.0, 30.0, 0.1, 0.5, 0.6, 0.01, paths=True)
            c = (time.perf_counter() - t1) / n
            res["cpu_baseline"] = {"value": c * 1e3, "unit": "ms per equilibrium", "cores": 1, "kind": "port",
                                   "host": host_info(), "sample": f"{n} single-point solves (learning + "
                                   "equilibrium + AW path) on one core"}
    else:
        g = sbr.fig5_grid(500)
        npts = g.n_points
        # the caller's result matrices, allocated once and refilled per call as the reference's
        # script fills its ξ / AW matrices (fresh 12 MB of host arrays per call cost page faults
        # that are the host allocator's, not the sweep's)
        host_out = {k: np.empty(npts) for k in sbr.engine.RESULT_FIELDS}
        host_out["status"] = np.empty(npts, np.uint32)
        host_out["iters"] = np.empty(npts, np.int32)
        for _ in range(max(a.warmup, 1)):
            r = eng.sweep_baseline(g, early_exit=5, out=host_out)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            r = eng.sweep_baseline(g, early_exit=5, out=host_out)
        dt = (time.perf_counter() - t0) / a.steps
        run = int(((r["status"] & sbr.STATUS["SBR_RUN"]) > 0).sum())
        # phase breakdown of one more call (events on the call's stream + host clock)
        eng.timing_enable(True)
        tp = time.perf_counter()
        eng.sweep_baseline(g, early_exit=5, out=host_out)
        py_call = (time.perf_counter() - tp) * 1e3
        phases = eng.host_phases()
        eng.timing_read(None)
        eng.timing_enable(False)
        phases["python_call"] = py_call
        res = {"metric": "equilibria solved/sec on β×u grid (FP64), Fig 5 500x500, one host-API call per grid",
               "value": npts / dt, "unit": "equilibria/s", "n_gpus": 1, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": None, "vs_baseline": None,
               "dtype": "f64", "data": "the reference's Fig 5 grid (deterministic)",
               "config": {"workload": "config2: sbr_sweep_baseline on fig5 500x500, early_exit_nan_run=5, host "
                                      "arrays (PCIe included) (BASELINE config 2)", "run_cells": run},
               "phase_ms": phases, "libsbr_sha16": lib_sha()}
        if not a.no_cpu_baseline:
            O.build()
            cores = usable_cores()
            t1 = time.perf_counter()
            o = O.sweep_baseline(g.beta, g.eta, g.t_end, g.u, g.p, g.kappa, g.lam, g.x0, nthreads=cores)
            O.apply_early_exit(o, 5)
            c = time.perf_counter() - t1
            res["cpu_baseline"] = {"value": npts / c, "unit": "equilibria/s", "cores": cores, "kind": "port",
                                   "host": host_info(), "sample": f"the whole 500x500 grid ({npts} points, every "
                                   f"point solved, 5-NaN rule as a post-pass like the GPU) in {c:.2f} s"}
    print(json.dumps(res), flush=True)


def main_multihost(a):
    """Config 3 (2048 x 2048) through the host-pointer C ABI on an n-device context
    (sbr_init_multi over every visible GPU, one process, one host thread per GPU): what a Julia
    ccall of sbr_sweep_baseline pays, PCIe included.  Reports the fan-out's phases: the slowest
    rank's sweep, its D2H into the pinned landing buffer, the host copy into the caller's arrays."""
    n_dev = torch.cuda.device_count()
    eng = sbr.Engine(n_gpus=n_dev)
    g = sbr.fig5_grid(a.n)
    npts = g.n_points
    host_out = {k: np.empty(npts) for k in sbr.engine.RESULT_FIELDS}
    host_out["status"] = np.empty(npts, np.uint32)
    host_out["iters"] = np.empty(npts, np.int32)
    for _ in range(max(a.warmup, 1)):
        eng.sweep_baseline(g, out=host_out)
    phases = []
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.sweep_baseline(g, out=host_out)
        phases.append(eng.host_phases())
    dt = (time.perf_counter() - t0) / a.steps
    mean = {k: float(np.mean([p[k] for p in phases])) for k in phases[0]}
    d2h_gbs = npts * 48 / n_dev / (mean["slowest_rank_d2h_pinned"] * 1e-3) / 1e9
    res = {"metric": "equilibria solved/sec on β×u grid (FP64), host-pointer n-device call (PCIe included)",
           "value": npts / dt, "unit": "equilibria/s", "n_gpus": n_dev, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": dt * 1e3, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "f64", "data": "the reference's Fig 5 grid at 2048 x 2048 (deterministic)",
           "config": {"workload": f"sbr_sweep_baseline on an sbr_init_multi({n_dev}) context, fig5 {a.n}x{a.n}, "
                                  "host arrays out, direct transport (pinned landing buffer per rank)",
                      "result_bytes_per_rank": npts * 48 // n_dev},
           "phase_ms_mean": mean, "d2h_GBps_per_rank": d2h_gbs, "libsbr_sha16": lib_sha()}
    print(json.dumps(res), flush=True)


def _unchanged_loop(lr, m, u_vals, nan_threshold=5):
    """scripts/1_baseline.jl's per-u loop body (Fig 4 :151-192, one Fig 5 column :231-262) through
    the Python mirror: ModelParameters(m; u=u), solve_equilibrium_baseline(lr, ·),
    get_AW_functions!, the 5-NaN early termination.  Returns (AW_max list, calls made)."""
    out, nan_run, calls = [], 0, 0
    for u in u_vals:
        if nan_run >= nan_threshold:
            out.extend([np.nan] * (len(u_vals) - len(out)))
            break
        m_u = sbr.ModelParameters.modify(m, u=float(u))
        r = sbr.solve_equilibrium_baseline(lr, m_u.economic)
        aw = sbr.get_AW_functions(r)
        calls += 1
        if r.bankrun:
            out.append(aw["AW_max"])
            nan_run = 0
        else:
            out.append(np.nan)
            nan_run += 1
    return out, calls


def main_dropin(a, eng, O):
    """The reference's scripts run unchanged on the drop-in (Python mirror of SBRDropIn.jl):
    Fig 4 = one solve_learning + 5,000 u of solve_equilibrium_baseline(lr, ·) + get_AW_functions!
    with the 5-NaN early exit (scripts/1_baseline.jl:137-192); each call solves on lr's own knots
    (sbr_equilibrium_on_knots: knots and HR resident, no learning ODE).  value = microseconds per
    solve_equilibrium_baseline + get_AW_functions! call, host API (PCIe round trip included).
    Also timed: the raw C-ABI call (Engine.equilibrium_on_knots with the paths) and the Fig 5
    500 x 500 loop (:210-267: 500 solve_learning + the per-u calls) end to end."""
    sbr.engine._default = eng
    m = sbr.ModelParameters.make(beta=1.0, eta_bar=15.0, u=0.1, p=0.5, kappa=0.6, lam=0.01)
    u4 = sbr.julia_range("0.001", "0.2", 5000)
    lr = sbr.solve_learning(m.learning)
    _unchanged_loop(lr, m, u4[:200])  # warm-up (first-call allocations)
    reps = max(a.steps // 10, 1)
    t0 = time.perf_counter()
    for _ in range(reps):
        aw4, calls4 = _unchanged_loop(lr, m, u4)
    dt4 = (time.perf_counter() - t0) / reps
    n_run4 = int(np.isfinite(aw4).sum())
    cdf = lr.learning_cdf
    k = 2000
    t1 = time.perf_counter()
    for j in range(k):
        eng.equilibrium_on_knots(cdf.knots, cdf.coefs, 1.0, 15.0, 30.0, float(u4[j % 2700]), 0.5, 0.6, 0.01)
    raw = (time.perf_counter() - t1) / k
    # Fig 5 unchanged: per β, ModelParameters(m_base; β=β), solve_learning, then the u loop
    amt = sbr.julia_range("0.0001", "1", 500)
    u5 = sbr.julia_range("0.001", "1", 500)
    t2 = time.perf_counter()
    calls5, learn5, run5 = 0, 0.0, 0
    for b in 1.0 / amt:
        m_b = sbr.ModelParameters.modify(m, beta=float(b))
        tl = time.perf_counter()
        lr_b = sbr.solve_learning(m_b.learning)
        learn5 += time.perf_counter() - tl
        col, c = _unchanged_loop(lr_b, m_b, u5)
        calls5 += c
        run5 += int(np.isfinite(col).sum())
    dt5 = time.perf_counter() - t2
    res = {"metric": "unchanged-script drop-in latency: solve_equilibrium_baseline(lr, econ) + get_AW_functions! "
                     "per call (Fig 4 loop, host API)",
           "value": dt4 / calls4 * 1e6, "unit": "us per call", "n_gpus": 1, "steps": reps, "warmup": 1,
           "ms_per_step": dt4 * 1e3, "higher_is_better": False, "scaling": None, "vs_baseline": None,
           "dtype": "f64", "data": "the reference's Fig 4 / Fig 5 grids (deterministic)",
           "config": {"workload": "scripts/1_baseline.jl Fig 4 loop (5000 u, 5-NaN early exit) through the Python "
                                  "mirror on one LearningResults (sbr_equilibrium_on_knots)"},
           "fig4": {"calls": calls4, "run_points": n_run4, "seconds": dt4},
           "raw_capi_us_per_call": raw * 1e6,
           "fig5_500_unchanged": {"seconds": dt5, "solve_learning_seconds": learn5, "calls": calls5,
                                  "run_points": run5, "us_per_call": (dt5 - learn5) / max(calls5, 1) * 1e6},
           "libsbr_sha16": lib_sha()}
    t3 = time.perf_counter()
    t_, G_, _ = O.learn_logistic(1.0, 30.0)
    n = 200
    for j in range(n):
        O.equilibrium_paths(t_, G_, 1.0, 15.0, 30.0, float(u4[j]), 0.5, 0.6, 0.01)
    c = (time.perf_counter() - t3 - 0.0) / n
    res["cpu_baseline"] = {"value": c * 1e6, "unit": "us per call", "cores": 1, "kind": "port", "host": host_info(),
                           "sample": f"{n} single-point solves on given knots (hazard + buffers + bisection + the "
                                     "three AW paths) on one core, plus one learning solve"}
    print(json.dumps(res), flush=True)


def main_launchcheck(a):
    """The launcher's plumbing without a GPU (tests/test_bench_launcher.py): every rank joins a
    gloo group on the MASTER_* rendezvous, the ranks' ids are summed, and rank 0 prints one line."""
    world, rank, _ = world_of(a.gpus)
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
        t = torch.tensor([rank], dtype=torch.int64)
        dist.all_reduce(t)
        rank_sum = int(t.item())
    else:
        rank_sum = 0
    if rank == 0:
        print(json.dumps({"workload": "launchcheck", "n_gpus": world, "rank_sum": rank_sum,
                          "parallelism": f"beta-column shards x{world}"}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    a = parse()
    if a.workload == "launchcheck":
        return main_launchcheck(a)
    if a.workload in ("config1", "config2", "dropin", "multihost"):
        return main_small(a)
    if a.workload == "social":
        return main_social(a)
    if a.workload == "hetero":
        return main_hetero(a)
    if a.workload == "interest":
        return main_interest(a)
    world, rank, local = world_of(a.gpus)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()

    n = a.n
    # weak (default): rank r owns columns r, r+N, … of a (n·N)-column grid; strong (--strong):
    # the n-column grid itself is dealt over the N ranks; --shard-of V: one process runs the
    # shard that rank --shard-rank of a V-rank strong run would own (a one-GPU rehearsal)
    rehearsal = a.shard_of > 1
    strong = a.strong or rehearsal
    if rehearsal and world != 1:
        raise SystemExit("bench.py: --shard-of rehearses one shard in one process (--gpus 1)")
    n_shards, shard = (a.shard_of, a.shard_rank) if rehearsal else (world, rank)
    if strong and n % n_shards:
        raise SystemExit(f"bench.py: --strong needs --n ({n}) divisible by the shard count ({n_shards})")
    n_axis = n if strong else n * world
    amt = sbr.julia_range("0.0001", "1", n_axis)
    cols = np.arange(shard, n_axis, n_shards)
    beta_h = 1.0 / amt[cols]
    u_h = sbr.julia_range("0.001", "1", n)
    nb, nu = len(beta_h), len(u_h)
    p, kappa, lam, x0 = 0.5, 0.6, 0.01, 1e-4

    pipe = not a.no_pipeline
    nbat = max(a.steps, a.warmup, 1) if pipe else 1
    # one row per batch (= step); every batch is the full config-3 grid, recomputed
    beta = torch.from_numpy(beta_h).to(dev).repeat(nbat, 1)
    eta = torch.full((nbat, nb), 15.0, dtype=torch.float64, device=dev)
    t_end = torch.full((nbat, nb), 30.0, dtype=torch.float64, device=dev)
    u = torch.from_numpy(u_h).to(dev)
    out = {k: torch.empty(nbat, nb * nu, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
    out["status"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nbat, nb * nu, dtype=torch.int32, device=dev)
    gather = world > 1 and not a.no_gather
    # the full SoA of every step, collected on rank k mod N (all-to-all per window of N steps)
    col = D.StepCollector(out, world, rank) if gather else None

    eng = sbr.Engine(local)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # a window's collection runs on its own stream as soon as its last step's results exist
    # (sbr_batch_wait), overlapped with the sweeps of the later steps
    comm = torch.cuda.Stream(dev) if gather and pipe else None

    if pipe and hasattr(eng._L, "sbr_batch_reserve"):
        # the batch's learning workspace for the longer of the warmup / timed calls, allocated
        # here (untimed) like the result tensors above
        eng.batch_reserve(nbat, nb)

    def run_steps(n):
        """n steps: one batch call of n grids (learned together, then the
        equilibria back to back); else one sweep call per step."""
        if n <= 0:
            return
        if pipe:
            eng.sweep_baseline_batch_dev(beta[:n], eta[:n], t_end[:n], u, p, kappa, lam, x0,
                                         {k: v[:n] for k, v in out.items()}, stream=stream)
            if gather:
                for k0, m in col.windows(n):
                    eng.batch_wait(comm.cuda_stream, k0 + m - 1)
                    with torch.cuda.stream(comm):
                        col.collect(k0, m)
        else:
            one = {k: v[0] for k, v in out.items()}
            for k in range(n):
                eng.sweep_baseline_dev(beta[0], eta[0], t_end[0], u, p, kappa, lam, x0, one, stream=stream,
                                       flags=sbr._lib.SBR_FLAG_READY_SWEEP if a.ready else 0)
                if gather:
                    col.collect(k, 1, row0=0)

    run_steps(a.warmup)
    torch.cuda.synchronize(dev)
    eng.timing_read(stream)  # drop anything recorded so far
    eng.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(a.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timeline = eng.chunk_timeline(stream) if not pipe else []  # the last sweep's chunk ends
    learn_ms, eq_ms, ncalls = eng.timing_read(stream)
    eng.timing_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- algorithmic flops of this rank's last step (from the kernels' own outputs) ----
    ls = eng.learn_stats(nb)
    last = (a.steps - 1) if pipe else 0
    iters = out["iters"][last].cpu().numpy().reshape(nb, nu).astype(np.int64)
    status = out["status"][last].cpu().numpy().view(np.uint32).reshape(nb, nu)
    run = (status & sbr.STATUS["SBR_RUN"]) > 0
    n_tau = ls["n_tau"].astype(np.int64)
    f_eq = (F8_BUFFER * nb * nu + F8_BISECT_ITER * int(iters.sum())
            + F8_AW_KNOT * int((run * n_tau[:, None]).sum()))
    f_learn = F8_RK_STEP * int((ls["n_accept"] + ls["n_reject"]).sum()) + F8_HZ_KNOT * int(n_tau.sum())
    # pipelined: narrow grids (strong-scaled shards) share learning and equilibrium launches
    # (libsbr groups them up to 2048 columns); the roofline is per launch, the kernel times per grid
    gpl = (a.steps / max(ncalls, 1)) if pipe else 1.0
    eq_s = eq_ms / max(ncalls, 1) / 1e3

    total_pts = nb * nu * world  # every rank's shard (strong: the whole n x n grid)
    value = total_pts * a.steps / elapsed
    if rehearsal:
        workload = (f"fig5_beta_u_sweep_{n}x{n} strong-scaled: shard {shard} of {n_shards} ({nb} beta columns x "
                    f"{nu} u) on one GPU, the per-GPU work of a {n_shards}-GPU run (BASELINE config 3)")
    elif strong:
        workload = f"fig5_beta_u_sweep_{n}x{n}_total strong-scaled over {world} GPU(s) (BASELINE config 3)"
    else:
        workload = f"fig5_beta_u_sweep_{n}x{n}_per_gpu (BASELINE config 3)"
    res = {
        "metric": "equilibria solved/sec on β×u grid (FP64)",
        "value": value,
        "unit": "equilibria/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic Fig 5 parameter grid; no RNG in the reference)",
        "config": {
            "workload": workload,
            "n_beta_per_gpu": nb, "n_u": nu, "eta": 15.0, "t_end": 30.0, "p": p, "kappa": kappa,
            "lambda": lam, "x0": x0, "early_exit": False,
            "collect": ("full SoA (48 B/pt) of every step on rank k mod N, all-to-all per N steps"
                        if gather else None),
            "parallelism": f"beta-column shards x{world}",
            "beta_axis_columns": n_axis,
            "pipelined": pipe,
            "single_sweep_schedule": None if pipe else ("per-column readiness" if a.ready else "chunked"),
        },
        # pipelined: per-launch kernel times (HIP events around each launch on its stream);
        # single sweep: libsbr cuts the grid into column chunks whose kernels overlap, so the
        # events give the learning stage's wall time and the equilibrium tail after it
        "kernel_ms_per_step": ({"learn_logistic": learn_ms / a.steps, "equilibrium": eq_ms / a.steps,
                                "equilibrium_launches": ncalls, "grids_per_launch": gpl}
                               if pipe else
                               {"learning_stage_wall": learn_ms / max(ncalls, 1),
                                "equilibrium_tail_after_learning": eq_ms / max(ncalls, 1)}
                               if not a.ready else
                               {"learn_logistic": learn_ms / max(ncalls, 1),
                                "eq_ready_concurrent": eq_ms / max(ncalls, 1)}),
        "flops_per_step": {"equilibrium": f_eq, "learn": f_learn},
        "work_per_step": {"run_points": int(run.sum()), "bisect_iters": int(iters.sum()),
                          "aw_knots_run": int((run * n_tau[:, None]).sum()),
                          "rk_steps": int((ls["n_accept"] + ls["n_reject"]).sum())},
        "roofline": (roofline("equilibrium_kernel", f_eq * gpl, eq_s, pmc_of("equilibrium_kernel<768, false, 1>",
                                                                   "-" if strong else f"fig5_{n}x{n}"))
                     if pipe else None),
        "libsbr_sha16": lib_sha(),
    }
    if not pipe:
        res["roofline_note"] = "single-sweep mode: chunked kernels overlap; the roofline line is the pipelined default run's"
        res["chunk_timeline_ms"] = [{"learn_end": a, "eq_end": b} for a, b in timeline]
    if a.phases:
        res["eq_phase_ms"] = phase_breakdown(eng, beta[0], eta[0], t_end[0], u, p, kappa, lam, x0,
                                             {k: v[0] for k, v in out.items()}, stream, dev)
    # the timed results checked against the oracle (test infrastructure, after the timed region):
    # the cpu_baseline leg's columns (every cpu_stride-th, all u) or 12 sampled columns
    oracle_cols = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        res["cpu_baseline"], oracle_cols, o_res = cpu_baseline(beta_h, u_h, a.cpu_stride, p, kappa, lam, x0)
    elif not a.no_verify:
        oracle_cols = np.sort(np.random.default_rng(rank).choice(nb, min(12, nb), replace=False))
        o_res = oracle_sweep(beta_h[oracle_cols], u_h, p, kappa, lam, x0)
    if oracle_cols is not None:
        res["verified"] = verify_grid(out, last, nb, nu, oracle_cols, o_res)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def oracle_sweep(beta_cols, u_h, p, kappa, lam, x0, nthreads=0):
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle as O  # noqa: E402  (test infrastructure: verification leg only)

    O.build()
    return O.sweep_baseline(beta_cols, 15.0, 30.0, u_h, p, kappa, lam, x0=x0, nthreads=nthreads or usable_cores())


def same_results(g: dict, o: dict, int_fields=("iters",)) -> bool:
    """Every float result field equal bit for bit (NaN where NaN), the status bits and the
    integer counters `int_fields` identical; g: GPU arrays, o: the oracle's, same shape."""
    ok = True
    for f in sbr.engine.RESULT_FIELDS:
        a, b = np.asarray(g[f]), np.asarray(o[f])
        ok &= a.shape == b.shape and bool(np.all((a == b) | (np.isnan(a) & np.isnan(b))))
    ok &= bool(np.array_equal(np.asarray(g["status"]).view(np.uint32), np.asarray(o["status"]).view(np.uint32)))
    for f in int_fields:
        ok &= bool(np.array_equal(np.asarray(g[f]).astype(np.int64), np.asarray(o[f]).astype(np.int64)))
    return bool(ok)


def verify_grid(out, k, nb, nu, cols, o) -> dict:
    """Grid k of the timed run (the last timed step) against the oracle on columns `cols`:
    every result field, status bit and bisection count, bit for bit."""
    ok = True
    for f in sbr.engine.RESULT_FIELDS:
        g = out[f][k].view(nb, nu)[torch.as_tensor(cols, device=out[f].device)].cpu().numpy()
        ok &= bool(np.all((g == o[f]) | (np.isnan(g) & np.isnan(o[f]))))
    st = out["status"][k].view(nb, nu)[torch.as_tensor(cols, device=out["status"].device)].cpu().numpy()
    ok &= bool(np.array_equal(st.view(np.uint32), o["status"]))
    it = out["iters"][k].view(nb, nu)[torch.as_tensor(cols, device=out["iters"].device)].cpu().numpy()
    ok &= bool(np.array_equal(it, o["iters"]))
    return {"bitwise_equal_oracle": ok, "grid": "last timed step", "columns": int(len(cols)),
            "points": int(len(cols) * nu)}


def main_hetero(a):
    """BASELINE config 4 (concretised in SURVEY.md §8(d), sbr.grids.hetero_config4): K = 8
    learning groups, βs_k = s·0.125·100^((k−1)/7), dist_k = 1/8, s = 1/range(1e-3, 1, n·N),
    u = range(0.001, 1, n), η = η_bar/Σdist·βs per column, tspan carried from s = 1.
    Weak scaling: rank r owns columns r, r+N, …  One step = learning (K-group Tsit5 +
    K hazards) for every column and buffers + ξ bisection + validity check + AW_max for
    every (column, u)."""
    world, rank, local = world_of(a.gpus)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
    n = a.hetero_n
    full = sbr.hetero_config4(n * world, n, K=8)
    g = full.subset(np.arange(rank, n * world, world))
    nb, nu, K = g.betas.shape[0], len(g.u), g.K
    betas = torch.from_numpy(np.ascontiguousarray(g.betas)).to(dev)
    distw = torch.from_numpy(g.dist).to(dev)
    eta = torch.from_numpy(np.ascontiguousarray(g.eta)).to(dev)
    t_end = torch.from_numpy(np.ascontiguousarray(g.t_end)).to(dev)
    u = torch.from_numpy(g.u).to(dev)
    out = {k: torch.empty(nb * nu, dtype=torch.float64, device=dev) for k in ("xi", "aw_max", "tol")}
    out["status"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    eng = sbr.Engine(local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    gather = world > 1 and not a.no_gather

    pipe = not a.no_pipeline
    nbat = max(a.steps, a.warmup, 1) if pipe else 1
    if pipe:  # one row per batch (= step), every batch the full per-rank grid, recomputed
        out_b = {k: torch.empty(nbat, nb * nu, dtype=v.dtype, device=dev) for k, v in out.items()}
        betas_b = betas.unsqueeze(0).repeat(nbat, 1, 1).contiguous()
        eta_b = eta.unsqueeze(0).repeat(nbat, 1).contiguous()
        t_end_b = t_end.unsqueeze(0).repeat(nbat, 1).contiguous()
    # every step's result SoA (ξ, AW_max, tol, status, iterations) on rank k mod N
    col = D.StepCollector(out_b if pipe else {k: v[None] for k, v in out.items()}, world, rank) if gather else None

    def run_steps(m):
        """m steps: pipelined, one batch call of m grids (learning of step k+1 overlaps the
        equilibrium of step k); else one sweep call per step."""
        if m <= 0:
            return
        if pipe:
            eng.sweep_hetero_batch_dev(K, betas_b[:m], distw, eta_b[:m], t_end_b[:m], u, g.p, g.kappa, g.lam, g.x0,
                                       {k: v[:m] for k, v in out_b.items()}, stream=stream)
            if gather:
                for k0, mm in col.windows(m):
                    col.collect(k0, mm)
            out["status"].copy_(out_b["status"][m - 1])
        else:
            for k in range(m):
                eng.sweep_hetero_dev(K, betas, distw, eta, t_end, u, g.p, g.kappa, g.lam, g.x0, out, stream=stream)
                if gather:
                    col.collect(k, 1, row0=0)

    run_steps(a.warmup)
    torch.cuda.synchronize(dev)
    eng.timing_read(stream)
    eng.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    run_steps(a.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    learn_ms, eq_ms, ncalls = eng.timing_read(stream)
    eng.timing_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = out["status"].cpu().numpy().view(np.uint32)
    # §8(d)-style algorithmic flops of the equilibrium kernel (batch 0 = learning slot 0):
    # K buffers, K-group bisection iterations, AW over the whole knot grid on run points
    # (get_AW_hetero); the validity check is not counted (a lower bound)
    hs = eng.hetero_learn_stats(nb)
    it_h = (out_b["iters"][0] if pipe else out["iters"]).cpu().numpy().reshape(nb, nu).astype(np.int64)
    st0 = (out_b["status"][0] if pipe else out["status"]).cpu().numpy().view(np.uint32).reshape(nb, nu)
    run_h = (st0 & sbr.STATUS["SBR_RUN"]) > 0
    nk_h = hs["n_knots"].astype(np.int64)
    f_eq_h = K * (F8_BUFFER * nb * nu + F8_BISECT_ITER * int(it_h.sum()) + F8_AW_KNOT * int((run_h * nk_h[:, None]).sum()))
    res = {
        "metric": "equilibria solved/sec on β×u grid (FP64), heterogeneity extension K=8",
        "value": nb * nu * world * a.steps / elapsed,
        "unit": "equilibria/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (deterministic config-4 parameter grid; no RNG in the reference)",
        "config": {"workload": f"hetero_K8_{nb}x{nu}_per_gpu (BASELINE config 4)", "n_col_per_gpu": nb,
                   "n_u": nu, "K": K, "eta_bar": 30.0, "p": g.p, "kappa": g.kappa, "lambda": g.lam,
                   "parallelism": f"column shards x{world}", "pipelined": pipe},
        "kernel_ms_per_step": {"learn_hetero": learn_ms / max(ncalls, 1), "equilibrium_hetero": eq_ms / max(ncalls, 1)},
        "run_fraction": float(((st & sbr.STATUS["SBR_RUN"]) > 0).mean()),
        # columns whose AutoSwitch moved to Rosenbrock23 (handled: restated in the engine and the oracle)
        "stiff_switch_fraction": float(((st & sbr.STATUS["SBR_STIFF_SWITCH"]) > 0).mean()),
        "stiff_switch": "handled (Rosenbrock23 restated, DESIGN.md §2)",
        "learn_steps_per_column": float((hs["n_accept"] + hs["n_reject"]).mean()),
        "roofline": roofline("equilibrium_hetero_kernel", f_eq_h, eq_ms / max(ncalls, 1) / 1e3,
                             pmc_of("equilibrium_hetero_kernel<8, 256, 1>", f"hetero_K8_{n}x{n}")),
        "libsbr_sha16": lib_sha(),
    }
    if a.phases:
        from sbr import _lib
        ph = {}
        for name, fl in (("scans", 0x100), ("bisect", 0x200), ("validity", 0x400), ("full", 0)):
            eng.sweep_hetero_dev(K, betas, distw, eta, t_end, u, g.p, g.kappa, g.lam, g.x0, out, stream=stream,
                                 flags=fl)
            torch.cuda.synchronize(dev)
            eng.timing_read(stream)
            eng.timing_enable(True)
            eng.sweep_hetero_dev(K, betas, distw, eta, t_end, u, g.p, g.kappa, g.lam, g.x0, out, stream=stream,
                                 flags=fl)
            torch.cuda.synchronize(dev)
            _, e_ms, nc = eng.timing_read(stream)
            eng.timing_enable(False)
            ph[name] = e_ms / max(nc, 1)
        res["eq_phase_ms"] = ph
    # the cpu_baseline leg's columns (every 16th) double as the check of the timed results: the
    # last timed grid against the oracle, bit for bit (test infrastructure, after the timed region)
    o_cols = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        o_cols = np.arange(0, nb, 16)
    elif not a.no_verify:
        o_cols = np.sort(np.random.default_rng(rank).choice(nb, min(4, nb), replace=False))
    if o_cols is not None:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle as O  # noqa: E402  (test infrastructure: cpu_baseline / verification leg only)

        O.build()
        cores = usable_cores()
        sub = g.subset(o_cols)
        t1 = time.perf_counter()
        o_h = O.sweep_hetero(sub.betas, sub.dist, sub.eta, sub.t_end, sub.u, sub.p, sub.kappa, sub.lam, sub.x0,
                             nthreads=cores)
        dt = time.perf_counter() - t1
        pts = sub.betas.shape[0] * nu
        if not a.no_cpu_baseline and rank == 0 and world == 1:
            res["cpu_baseline"] = {"value": pts / dt, "unit": "equilibria/s", "cores": cores, "kind": "port",
                                   "host": host_info(),
                                   "sample": f"{sub.betas.shape[0]} columns (every 16th) x {nu} u = {pts} equilibria "
                                             f"in {dt:.2f} s"}
        last = (out_b if pipe else {k: v[None] for k, v in out.items()})
        k_last = (a.steps - 1) if pipe else 0
        idx = torch.as_tensor(o_cols, device=dev)
        ok = True
        for f in ("xi", "aw_max", "tol"):
            gv = last[f][k_last].view(nb, nu)[idx].cpu().numpy()
            ok &= bool(np.all((gv == o_h[f]) | (np.isnan(gv) & np.isnan(o_h[f]))))
        stv = last["status"][k_last].view(nb, nu)[idx].cpu().numpy().view(np.uint32)
        ok &= bool(np.array_equal(stv, o_h["status"]))
        itv = last["iters"][k_last].view(nb, nu)[idx].cpu().numpy()
        ok &= bool(np.array_equal(itv, o_h["iters"]))
        res["verified"] = {"bitwise_equal_oracle": ok, "grid": "last timed step", "columns": int(len(o_cols)),
                           "points": int(pts)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_interest(a):
    """Interest-rate extension (interest_rate_solver.jl:51-150, value_function_solver.jl:66-112)
    on the Fig 5 grid shape: β = 1/range(1e-4, 1, n·N) (η = 15, tspan (0, 30) carried),
    u = range(0.001, 1, n), p = 0.5, κ = 0.6, λ = 0.01 and scripts/3_interest_rates.jl's
    r = 0.06, δ = 0.1.  Weak scaling over β columns.  One step = learning + hazard per
    column and, per (β, u), the value-function Tsit5 solve on the HR grid, the buffers
    on h − rV, the ξ bisection and AW_max."""
    world, rank, local = world_of(a.gpus)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
    n = a.interest_n
    beta_all = 1.0 / sbr.julia_range("0.0001", "1", n * world)
    beta_h = np.ascontiguousarray(beta_all[rank::world])
    u_h = sbr.julia_range("0.001", "1", n)
    nb, nu = len(beta_h), len(u_h)
    r_, delta, p, kappa, lam, x0 = 0.06, 0.1, 0.5, 0.6, 0.01, 1e-4
    beta = torch.from_numpy(beta_h).to(dev)
    eta = torch.full((nb,), 15.0, dtype=torch.float64, device=dev)
    t_end = torch.full((nb,), 30.0, dtype=torch.float64, device=dev)
    u = torch.from_numpy(u_h).to(dev)
    out = {k: torch.empty(nb * nu, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
    out["status"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["rk_steps"] = torch.empty(nb * nu, dtype=torch.int64, device=dev)
    eng = sbr.Engine(local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    gather = world > 1 and not a.no_gather
    col = D.StepCollector({k: v[None] for k, v in out.items()}, world, rank) if gather else None
    n_done = [0]

    def step():
        eng.sweep_interest_dev(beta, eta, t_end, u, p, kappa, lam, r_, delta, x0, out, stream=stream)
        if gather:  # the step's full result SoA on rank (step mod N)
            col.collect(n_done[0], 1, row0=0)
        n_done[0] += 1

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)
    eng.timing_read(stream)
    eng.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    learn_ms, eq_ms, ncalls = eng.timing_read(stream)
    eng.timing_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    st = out["status"].cpu().numpy().view(np.uint32)
    steps = out["rk_steps"].cpu().numpy()
    ls = eng.learn_stats(nb)
    it_i = out["iters"].cpu().numpy().reshape(nb, nu).astype(np.int64)
    run_i = ((st & sbr.STATUS["SBR_RUN"]) > 0).reshape(nb, nu)
    nt_i = ls["n_tau"].astype(np.int64)
    # §8(d) flops of the interest kernel: the value-function Tsit5 steps, then the baseline's
    # buffers / bisection / AW path (the h − rV scan is not counted: a lower bound)
    f_eq_i = (F8_RK_STEP * int(steps.sum()) + F8_BUFFER * nb * nu + F8_BISECT_ITER * int(it_i.sum())
              + F8_AW_KNOT * int((run_i * nt_i[:, None]).sum()))
    res = {
        "metric": "equilibria solved/sec on β×u grid (FP64), interest-rate extension (value function per point)",
        "value": nb * nu * world * a.steps / elapsed,
        "unit": "equilibria/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (deterministic Fig-5-shaped parameter grid; no RNG in the reference)",
        "config": {"workload": f"interest_fig5_{nb}x{nu}_per_gpu (extension, SURVEY.md §8(f) rank 2)",
                   "n_beta_per_gpu": nb, "n_u": nu, "r": r_, "delta": delta, "eta": 15.0, "t_end": 30.0, "p": p,
                   "kappa": kappa, "lambda": lam, "parallelism": f"beta-column shards x{world}"},
        "kernel_ms_per_step": {"learn_logistic": learn_ms / max(ncalls, 1), "interest_equilibrium": eq_ms / max(ncalls, 1)},
        "value_fn_rk_steps_per_point": float(steps.mean()),
        "run_fraction": float(((st & sbr.STATUS["SBR_RUN"]) > 0).mean()),
        "stiff_switch_fraction": float(((st & sbr.STATUS["SBR_STIFF_SWITCH"]) > 0).mean()),
        "roofline": roofline("equilibrium_kernel<*, true> (interest)", f_eq_i, eq_ms / max(ncalls, 1) / 1e3,
                             pmc_of("equilibrium_kernel<512, true, 1>", f"interest_fig5_{n}x{n}")),
        "libsbr_sha16": lib_sha(),
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle as O  # noqa: E402  (test infrastructure: cpu_baseline leg only)

        O.build()
        cores = usable_cores()
        sub = beta_h[::10]
        t1 = time.perf_counter()
        o_i = O.sweep_interest(sub, 15.0, 30.0, u_h, p, kappa, lam, r_, delta, nthreads=cores)
        dt = time.perf_counter() - t1
        pts = len(sub) * nu
        res["cpu_baseline"] = {"value": pts / dt, "unit": "equilibria/s", "cores": cores, "kind": "port",
                               "host": host_info(),
                               "sample": f"{len(sub)} columns (every 10th) x {nu} u = {pts} equilibria "
                                         f"in {dt:.2f} s"}
        # the sample's points of the last timed sweep against the oracle, bit for bit
        gv = {k: v.view(nb, nu)[::10].cpu().numpy() for k, v in out.items()}
        res["verified"] = dict(bitwise_equal_oracle=same_results(gv, o_i, ("iters", "rk_steps")),
                               grid="last timed step", columns=len(sub), points=pts,
                               fields="xi, tau_in_unc, tau_out_unc, aw_max, tol, status, iters, rk_steps")
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_social(a):
    """BASELINE config 5: the social-learning fixed point (social_learning_solver.jl:63-263,
    tol 1e-4, max_iter 500 as in scripts/4_social_learning.jl:55) on β = 1/range(0.01, 2, 512)
    × u = range(0.001, 1, 512) with m_social's other parameters (η = 30/0.9 carried).  Weak
    scaling: rank r owns β columns r, r+N, … of a (cols·N)-column grid; cols = 64 makes N = 8
    exactly the 512×512 config.  One step = the whole fixed point for every point."""
    world, rank, local = world_of(a.gpus)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
    ncol = a.social_cols * world
    # the config-5 β axis (512 columns); fewer ranks take an evenly strided share of it
    n_axis = max(512, ncol)
    stride = n_axis // ncol if n_axis % ncol == 0 else 1
    amt = sbr.julia_range("0.01", "2", n_axis)
    cols = np.arange(rank, ncol, world) * stride
    beta_h = 1.0 / amt[cols]
    u_h = sbr.julia_range("0.001", "1", 512)
    eta_v = 30.0 / 0.9
    nb, nu = len(beta_h), len(u_h)
    p, kappa, lam, x0, tol = 0.99, 0.25, 0.25, 1e-4, 1e-4
    cmp_h = np.stack([sbr.julia_range(0.0, eta_v, 1000)] * nb)
    beta = torch.from_numpy(beta_h).to(dev)
    eta = torch.full((nb,), eta_v, dtype=torch.float64, device=dev)
    u = torch.from_numpy(u_h).to(dev)
    cmp = torch.from_numpy(cmp_h).to(dev)
    out = {k: torch.empty(nb * nu, dtype=torch.float64, device=dev) for k in sbr.engine.RESULT_FIELDS}
    out["status"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["iters"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["fp_iters"] = torch.empty(nb * nu, dtype=torch.int32, device=dev)
    out["rk_steps"] = torch.empty(nb * nu, dtype=torch.int64, device=dev)
    eng = sbr.Engine(local)
    stream = torch.cuda.current_stream(dev).cuda_stream
    gather = world > 1 and not a.no_gather
    col = D.StepCollector({k: v[None] for k, v in out.items()}, world, rank) if gather else None
    n_done = [0]

    flags = sbr._lib.SBR_FLAG_DIAG_SOCIAL_PROF if a.social_prof else 0

    def step():
        eng.sweep_social_dev(beta, eta, u, p, kappa, lam, cmp, x0, out, tol=tol, max_iter=a.social_max_iter,
                             stream=stream, flags=flags)
        if gather:  # the step's full result SoA on rank (step mod N)
            col.collect(n_done[0], 1, row0=0)
        n_done[0] += 1

    for _ in range(a.warmup):
        step()
    if a.warmup == 0:
        # one untimed single-iterate sweep of the same grid: sizes the knot workspaces and has the
        # driver clear their pages (≈2 s in a process that follows another on the box), which is
        # allocation, not part of solving a share
        eng.sweep_social_dev(beta, eta, u, p, kappa, lam, cmp, x0, out, tol=tol, max_iter=1, stream=stream)
    torch.cuda.synchronize(dev)
    eng.timing_read(stream)
    eng.timing_enable(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    init_ms, iter_ms, ncalls = eng.timing_read(stream)
    eng.timing_enable(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    steps = out["rk_steps"].cpu().numpy()
    st = out["status"].cpu().numpy().view(np.uint32)
    fp = out["fp_iters"].cpu().numpy()
    if a.social_dump:
        np.savez(a.social_dump, beta=beta_h, u=u_h, status=st, fp_iters=fp, rk_steps=steps,
                 xi=out["xi"].cpu().numpy(), aw_max=out["aw_max"].cpu().numpy())
    total_pts = nb * nu * world
    res = {
        "metric": "equilibria solved/sec on β×u grid (FP64), social-learning fixed point",
        "value": total_pts * a.steps / elapsed,
        "unit": "equilibria/s",
        "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (deterministic config-5 parameter grid; no RNG in the reference)",
        "config": {"workload": f"social_fixed_point_{nb}x{nu}_per_gpu (BASELINE config 5 share)",
                   "n_beta_per_gpu": nb, "n_u": nu, "eta": eta_v, "p": p, "kappa": kappa, "lambda": lam,
                   "tol": tol, "max_iter": a.social_max_iter, "parallelism": f"beta-column shards x{world}"},
        "kernel_ms_per_step": {"social_init": init_ms / max(a.steps, 1), "social_iterates": iter_ms / max(a.steps, 1)},
        "passes_per_step": ncalls / max(a.steps, 1),
        "knot_overflow": eng.social_overflow_stats(),
        "rk_steps_per_point": float(steps.mean()),
        "fp_iters_mean": float(fp.mean()), "fp_iters_max": int(fp.max()),
        "run_fraction": float(((st & sbr.STATUS["SBR_RUN"]) > 0).mean()),
        "not_converged_fraction": float(((st & sbr.STATUS["SBR_SOCIAL_NOT_CONVERGED"]) > 0).mean()),
        "stiff_switch_fraction": float(((st & sbr.STATUS["SBR_STIFF_SWITCH"]) > 0).mean()),
        # §8(d) flops of the forced-ODE steps only (96 per attempted step; the per-iterate
        # hazard / bisection / AW / norm work is not counted: a lower bound), over the
        # whole share's wall time of the iterate kernels
        "roofline": roofline("social_iter_kernel", F8_RK_STEP * float(steps.sum()), iter_ms / max(a.steps, 1) / 1e3,
                             pmc_social(float(steps.sum()))),
        "libsbr_sha16": lib_sha(),
    }
    if res["roofline"]["traffic"] is not None:
        res["roofline"]["traffic_note"] = ("HBM bytes of the whole share: the PMC run's bytes per attempted RK step "
                                           "(first 16 iterates of the share, tools/pmc_social.py) x this run's RK steps; "
                                           "executed flops count 64 lanes per wave instruction (an upper bound)")
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle as O  # noqa: E402  (test infrastructure: cpu_baseline leg only)

        O.build()
        cores = usable_cores()
        # 16 β x 4 u = 64 points spread over the share (dynamic scheduling over points on every
        # usable core).  The share's cost is dominated by a few long fixed points, so the rate is
        # normalised by work: the sample's RK steps per second over the share's mean RK steps per
        # point (from this run's own per-point counts), next to the raw sample rate.
        bsel, usel = beta_h[::4], u_h[::128]
        t1 = time.perf_counter()
        cs = O.sweep_social(bsel, eta_v, usel, p, kappa, lam, cmp_h[: len(bsel)], x0=x0, tol=tol,
                            max_iter=a.social_max_iter, nthreads=cores, stats=True)
        dt = time.perf_counter() - t1
        pts = len(bsel) * len(usel)
        cpu_steps = float((cs["n_accept"] + cs["n_reject"]).sum())
        grid_steps = float(steps.mean())
        # the sample's fixed points of the timed sweep against the oracle, bit for bit
        gv = {k: v.view(nb, nu)[::4, ::128].cpu().numpy() for k, v in out.items()}
        res["verified"] = dict(bitwise_equal_oracle=same_results(gv, cs, ("iters", "fp_iters")),
                               grid="the timed sweep", points=pts,
                               fields="xi, tau_in_unc, tau_out_unc, aw_max, tol, status, iters, fp_iters")
        res["cpu_baseline"] = {"value": (cpu_steps / dt) / grid_steps, "unit": "equilibria/s", "cores": cores,
                               "kind": "port", "host": host_info(),
                               "raw_sample_rate": pts / dt,
                               "sample": f"{len(bsel)} β (every 4th) x {len(usel)} u (every 128th) = {pts} "
                                         f"fixed points in {dt:.2f} s ({cpu_steps:.3e} RK steps); value = sample RK "
                                         f"steps/s over the share's mean {grid_steps:.3e} RK steps per point"}
    if a.social_prof:
        pr = eng.social_prof_read()
        names = ("cmp_prelude", "ode", "hazard_scan", "bisection", "aw_norm", "damping_awmax")
        tot = max(sum(pr[:6]), 1)
        res["social_prof"] = {"cycle_share": {k: pr[i] / tot for i, k in enumerate(names)},
                              "cycles_per_rk_step_ode": pr[1] / max(pr[7], 1),
                              "slow_lookups_per_step": pr[6] / max(pr[7], 1)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def phase_breakdown(eng, beta, eta, t_end, u, p, kappa, lam, x0, out, stream, dev, reps=3):
    """Equilibrium-kernel time when every point stops after the crossing scan,
    after the bisection, and in full; plus AW knots evaluated exactly per run point.  Runs
    through the batch entry point with one grid: its timing events bracket the
    equilibrium launch itself (a single sweep is chunked, see kernel_ms_per_step)."""
    from sbr import _lib
    res = {}
    b2, e2, t2 = beta[None, :], eta[None, :], t_end[None, :]
    o2 = {k: v[None, :] for k, v in out.items()}

    class _One:  # sweep_baseline_dev-shaped adapter over the one-grid batch call
        @staticmethod
        def sweep_baseline_dev(beta, eta, t_end, u, p, kappa, lam, x0, out, stream=None, exhaustive=False, flags=0):
            fl = flags | (_lib.SBR_FLAG_EXHAUSTIVE if exhaustive else 0)
            eng.sweep_baseline_batch_dev(b2, e2, t2, u, p, kappa, lam, x0, o2, stream=stream, flags=fl)
    eng_one = _One()
    for name, fl in (("buffer", _lib.SBR_FLAG_DIAG_STOP_AFTER_BUFFER), ("bisect", _lib.SBR_FLAG_DIAG_STOP_AFTER_BISECT),
                     ("full", 0), ("full_exhaustive_aw", -1)):
        kw = dict(exhaustive=True) if fl == -1 else dict(flags=fl)
        eng_one.sweep_baseline_dev(beta, eta, t_end, u, p, kappa, lam, x0, out, stream=stream, **kw)
        torch.cuda.synchronize(dev)
        eng.timing_read(stream)
        eng.timing_enable(True)
        for _ in range(reps):
            eng_one.sweep_baseline_dev(beta, eta, t_end, u, p, kappa, lam, x0, out, stream=stream, **kw)
        torch.cuda.synchronize(dev)
        _, eq_ms, nc = eng.timing_read(stream)
        eng.timing_enable(False)
        res[name] = eq_ms / max(nc, 1)
    eng_one.sweep_baseline_dev(beta, eta, t_end, u, p, kappa, lam, x0, out, stream=stream,
                               flags=_lib.SBR_FLAG_DIAG_COUNT_AW_BLOCKS)
    torch.cuda.synchronize(dev)
    st = out["status"].cpu().numpy().view(np.uint32)
    nb = out["iters"].cpu().numpy()[(st & sbr.STATUS["SBR_RUN"]) > 0]
    res["aw_knots_evaluated_per_run_point"] = float(nb.mean()) if nb.size else 0.0
    res["run_points"] = int(nb.size)
    return res


def cpu_baseline(beta_h, u_h, stride, p, kappa, lam, x0):
    """The CPU oracle (C restatement, same algorithm, OpenMP over β columns) on a
    bounded sample of the same workload: every `stride`-th β column, all u.  Returns the
    baseline block, the sampled column indices and the oracle's results on them."""
    cores = usable_cores()
    idx = np.arange(0, len(beta_h), stride)
    cols = beta_h[idx]
    oracle_sweep(cols[:1], u_h[:4], p, kappa, lam, x0, nthreads=1)  # build / load outside the clock
    t0 = time.perf_counter()
    o = oracle_sweep(cols, u_h, p, kappa, lam, x0, nthreads=cores)
    dt = time.perf_counter() - t0
    pts = len(cols) * len(u_h)
    return ({"value": pts / dt, "unit": "equilibria/s", "cores": cores, "kind": "port", "host": host_info(),
             "sample": f"{len(cols)} β columns (every {stride}th of the {len(beta_h)}) x {len(u_h)} u = {pts} "
                       f"equilibria in {dt:.2f} s"}, idx, o)


if __name__ == "__main__":
    main()
