#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc passes (tools/pmc.sh) into a per-kernel table.

Usage: python tools/pmc_summary.py gpurun_out/pmc profiles/rNN_pmc.txt [workload [profiles/pmc_latest.json]]

Every counter is averaged per dispatch of a kernel (summed over the device).
The optional JSON (merged per workload) holds every kernel's counters, its HBM
traffic per launch corrected as MI355X_MICROARCH.md's HBM section prescribes
(FETCH_SIZE (KiB) doubled on gfx950, WRITE_SIZE (KiB) as is) and the sha of the
kernel's machine code, for bench.py's roofline.traffic / frac_executed.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pmc_dir):
    # (kernel, counter) -> {dispatch_id: value}
    vals = defaultdict(dict)
    for path in sorted(glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"]
                vals[(k, row["Counter_Name"])][(path, row["Dispatch_Id"])] = float(row["Counter_Value"])
    return vals


def short(name):
    return name.split("(")[0].replace("void ", "").replace("sbr::", "")


def main():
    pmc_dir, out_txt = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "fig5_2048x2048"
    out_json = sys.argv[4] if len(sys.argv) > 4 else None
    vals = load(pmc_dir)
    kernels = sorted({k for k, _ in vals if not k.startswith("__amd")})
    lines = ["# per-dispatch averages of rocprofv3 --pmc passes (%s)" % pmc_dir]
    per = {}
    for k in kernels:
        lines.append("\n## " + short(k))
        per[k] = {}
        for (kk, c), d in sorted(vals.items()):
            if kk != k:
                continue
            avg = sum(d.values()) / len(d)
            per[k][c] = avg
            lines.append("  %-26s %14.4g   (%d dispatches)" % (c, avg, len(d)))
        c = per[k]
        if "SQ_WAVE_CYCLES" in c and "SQ_WAIT_ANY" in c:
            w = c["SQ_WAVE_CYCLES"]
            lines.append("  -> wait_any %.1f%%  issue_stall %.1f%%  active %.1f%% of wave cycles" % (
                100 * c["SQ_WAIT_ANY"] / w, 100 * c.get("SQ_WAIT_INST_ANY", 0) / w,
                100 * c.get("SQ_ACTIVE_INST_ANY", 0) / w))
        if "SQ_THREAD_CYCLES_VALU" in c and c.get("SQ_ACTIVE_INST_VALU"):
            lines.append("  -> VALU lane utilisation %.3f (SQ_THREAD_CYCLES_VALU / (SQ_ACTIVE_INST_VALU x 64))" % (
                c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"])))
        if "SQ_INSTS_SALU" in c and c.get("SQ_INSTS_VALU"):
            lines.append("  -> SALU share %.3f of VALU + SALU instructions" % (
                c["SQ_INSTS_SALU"] / (c["SQ_INSTS_SALU"] + c["SQ_INSTS_VALU"])))
        if c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0) > 0:
            lines.append("  -> L2 hit rate %.3f" % (c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])))
        if c.get("TCP_TOTAL_CACHE_ACCESSES_sum") and "TCP_TCC_READ_REQ_sum" in c:
            lines.append("  -> L1 (TCP) read requests reaching L2: %.3f of accesses" % (
                c["TCP_TCC_READ_REQ_sum"] / c["TCP_TOTAL_CACHE_ACCESSES_sum"]))
        if "FETCH_SIZE" in c:
            lines.append("  -> HBM read %.1f MB (FETCH_SIZE x2, gfx950)" % (2 * c["FETCH_SIZE"] * 1024 / 1e6))
        if "WRITE_SIZE" in c:
            lines.append("  -> HBM write %.1f MB" % (c["WRITE_SIZE"] * 1024 / 1e6))
    with open(out_txt, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    # per-kernel counter averages, each tagged with the sha of the kernel's gfx950 code in
    # libsbr.so (sbr.provenance): bench.py folds a kernel's counters into its roofline line
    # (traffic, frac_executed) only while that machine code is unchanged.  Merged per workload.
    if out_json:
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                        "replication-social-bank-runs_amd"))
        from sbr import provenance as P
        try:
            pm = json.load(open(out_json))
        except Exception:
            pm = {}
        if "workloads" not in pm:
            pm = {"workloads": {}}
        ks = {}
        for k in kernels:
            d = dict(per[k])
            d["code_sha16"] = P.kernel_code_sha(short(k)) if "sbr::" in k else None
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:  # MI355X_MICROARCH.md: FETCH_SIZE (KiB) x2 on gfx950
                d["hbm_read_bytes"] = 2 * d["FETCH_SIZE"] * 1024
                d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
                d["hbm_bytes_per_launch"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
            ks[short(k)] = d
        pm["workloads"][workload] = {"source": out_txt, "kernels": ks}
        with open(out_json, "w") as f:
            json.dump(pm, f, indent=1)


if __name__ == "__main__":
    main()
