#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc passes (tools/pmc.sh) into a per-kernel table.

Usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r01_v3_pmc.txt [profiles/traffic_latest.json [workload
       [profiles/pmc_latest.json]]]

Every counter is averaged per dispatch of a kernel (summed over the device).
The optional JSON holds HBM traffic per launch of the equilibrium kernel for
bench.py's roofline.traffic, corrected as MI355X_MICROARCH.md's HBM section
prescribes: FETCH_SIZE (KiB) doubled on gfx950, WRITE_SIZE (KiB) as is.
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
    out_json = sys.argv[3] if len(sys.argv) > 3 else None
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
        if "FETCH_SIZE" in c:
            lines.append("  -> HBM read %.1f MB (FETCH_SIZE x2, gfx950)" % (2 * c["FETCH_SIZE"] * 1024 / 1e6))
        if "WRITE_SIZE" in c:
            lines.append("  -> HBM write %.1f MB" % (c["WRITE_SIZE"] * 1024 / 1e6))
    with open(out_txt, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if out_json:
        eq = [k for k in kernels if "equilibrium_kernel" in k and "hetero" not in k]
        if eq:
            c = per[eq[0]]
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                t = {"kernel": short(eq[0]), "workload": sys.argv[4] if len(sys.argv) > 4 else "fig5_2048x2048",
                     "source": out_txt,
                     "read_bytes": 2 * c["FETCH_SIZE"] * 1024, "write_bytes": c["WRITE_SIZE"] * 1024}
                t["hbm_bytes_per_launch"] = t["read_bytes"] + t["write_bytes"]
                with open(out_json, "w") as f:
                    json.dump(t, f, indent=1)
    # per-kernel counter averages + the libsbr.so they were collected on (bench.py's
    # roofline.frac_executed uses them only for that exact binary)
    if len(sys.argv) > 5:
        import hashlib
        lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "replication-social-bank-runs_amd", "lib",
                           "libsbr.so")
        sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
        pm = {"workload": sys.argv[4], "source": out_txt, "libsbr_sha16": sha,
              "kernels": {short(k): per[k] for k in kernels}}
        with open(sys.argv[5], "w") as f:
            json.dump(pm, f, indent=1)


if __name__ == "__main__":
    main()
