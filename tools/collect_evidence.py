#!/usr/bin/env python3
"""Copy a GPU evidence run's results into profiles/: the bench JSON line of every
gpurun_out/<tag>/<step>.out as profiles/<prefix>_<step>.json, the pytest log and smoke
output as text, and each rocprofv3 kernel-stats CSV as profiles/<prefix>_<dir>_kernel_stats.csv.
  python3 tools/collect_evidence.py <tag> <prefix>"""
import json
import shutil
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def main():
    tag, prefix = sys.argv[1], sys.argv[2]
    src = REPO / "gpurun_out" / tag
    dst = REPO / "profiles"
    for f in sorted(src.glob("*.out")):
        lines = [l for l in f.read_text().splitlines() if l.startswith("{")]
        if f.stem == "tests":
            shutil.copy(f, dst / f"{prefix}_gpu_tests.txt")
        elif f.stem == "smoke":
            shutil.copy(f, dst / f"{prefix}_smoke.txt")
        elif lines:
            json.loads(lines[-1])
            (dst / f"{prefix}_{f.stem}.json").write_text(lines[-1] + "\n")
        else:
            continue
        print(f.stem)
    for d in sorted(src.iterdir()):
        ks = d / "run_kernel_stats.csv"
        if d.is_dir() and ks.exists():
            shutil.copy(ks, dst / f"{prefix}_{d.name}_kernel_stats.csv")
            print(d.name, "kernel stats")


if __name__ == "__main__":
    main()
