#!/usr/bin/env python3
"""Fold a social-sweep PMC run (tools/pmc.sh on `bench.py --workload social --social-max-iter 16`)
into profiles/pmc_latest.json, normalised per attempted RK step, so that bench.py's social line
can report traffic and frac_executed for a whole share.

The counters are summed over the run's dispatches of social_iter_kernel (not averaged: one share
is many launches), and divided by the run's total RK steps, which each pass's bench JSON line
records (rk_steps_per_point × points).  Usage:

    python tools/pmc_social.py gpurun_out/<tag>/pmc_socbulk [profiles/pmc_latest.json]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
WORKLOAD = "social_64x512_bulk16"
KERNEL = "social_iter_kernel"


def main():
    pmc_dir = sys.argv[1]
    out_json = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "pmc_latest.json")
    sums = defaultdict(float)
    counted = defaultdict(int)
    steps = None
    for p in sorted(glob.glob(os.path.join(pmc_dir, "p*"))):
        if not os.path.isdir(p):
            continue
        part = defaultdict(float)
        for path in glob.glob(os.path.join(p, "*counter_collection.csv")):
            with open(path) as f:
                for row in csv.DictReader(f):
                    if KERNEL in row["Kernel_Name"]:
                        part[row["Counter_Name"]] += float(row["Counter_Value"])
        log = p + ".log"
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{"):
                    d = json.loads(line)
                    n = d["config"]["n_beta_per_gpu"] * d["config"]["n_u"]
                    s = d["rk_steps_per_point"] * n
                    steps = s if steps is None else steps
        for c, v in part.items():  # a counter collected in two passes: the mean of the passes
            sums[c] += v
            counted[c] += 1
    if not steps:
        raise SystemExit("no RK step count found in the pass logs")
    tot = {c: sums[c] / counted[c] for c in sums}
    per = {c: v / steps for c, v in tot.items()}
    sys.path.insert(0, os.path.join(REPO, "replication-social-bank-runs_amd"))
    from sbr import provenance as P
    d = {"per_rk_step": per, "rk_steps_total": steps, "source": pmc_dir,
         "code_sha16": P.kernel_code_sha(KERNEL)}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:  # MI355X_MICROARCH.md: FETCH_SIZE (KiB) x2 on gfx950
        d["hbm_bytes_per_rk_step"] = 2 * per["FETCH_SIZE"] * 1024 + per["WRITE_SIZE"] * 1024
    if "SQ_INSTS_VALU_FMA_F64" in per:
        d["fp64_flops_executed_per_rk_step"] = 64 * (per.get("SQ_INSTS_VALU_ADD_F64", 0) + per.get("SQ_INSTS_VALU_MUL_F64", 0)
                                                     + per.get("SQ_INSTS_VALU_TRANS_F64", 0)) + 128 * per["SQ_INSTS_VALU_FMA_F64"]
    try:
        pm = json.load(open(out_json))
    except Exception:
        pm = {"workloads": {}}
    pm.setdefault("workloads", {})[WORKLOAD] = {"source": pmc_dir, "kernels": {KERNEL: d}}
    with open(out_json, "w") as f:
        json.dump(pm, f, indent=1)
    print(json.dumps({k: v for k, v in d.items() if k != "per_rk_step"}, indent=1))


if __name__ == "__main__":
    main()
