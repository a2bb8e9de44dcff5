"""Extract the reference's Julia call surface per script → tests/golden/julia_surface.json.

For each of scripts/1_baseline.jl … 4_social_learning.jl (all under /root/reference) this
records, with file:line, what the script needs from the files the drop-ins replace:
  * its includes, split into the files a drop-in replaces and the ones it keeps (parameter
    and result-struct files, plotting.jl);
  * every function defined in the replaced files (positional arity, keyword names);
  * every call the script — and the kept plotting.jl — makes to one of them (positional
    count, keywords used);
  * what each called function returns (the struct it constructs or the NamedTuple's keys);
  * the fields the script reads on the values those calls return, and the fields
    plotting.jl reads on `result::SolvedModel`;
  * the fields of every struct defined in the replaced files (the drop-ins must define them)
    and in the kept files (the drop-ins construct them).
tests/test_julia_shim.py checks the drop-ins (julia/SBRDropIn*.jl) against this file; the
image has no Julia, so the check is static.  Run: python tools/extract_julia_surface.py
"""
from __future__ import annotations

import json
import re
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "tests"))
import jl_surface as J  # noqa: E402

REF = Path("/root/reference")
OUT = REPO / "tests" / "golden" / "julia_surface.json"

# which included files each script keeps, and which drop-ins replace the rest
KEEP_PATTERNS = ("_model.jl", "/model.jl", "plotting.jl")
DROPINS = {
    "scripts/1_baseline.jl": ["SBRDropIn.jl"],
    "scripts/2_heterogeneity.jl": ["SBRDropIn.jl", "SBRDropInHetero.jl"],
    "scripts/3_interest_rates.jl": ["SBRDropIn.jl", "SBRDropInInterest.jl"],
    "scripts/4_social_learning.jl": ["SBRDropIn.jl", "SBRDropInSocial.jl"],
}


def includes(path: Path) -> list[Path]:
    """include(joinpath(@__DIR__, "..", …)) lines of a file, resolved, transitively."""
    out = []
    src = J.strip_comments(path.read_text())
    for m in re.finditer(r"include\(\s*joinpath\(\s*@__DIR__\s*,([^)]*)\)\s*\)", src):
        parts = [p.strip().strip('"') for p in m.group(1).split(",")]
        f = (path.parent.joinpath(*parts)).resolve()
        out.append(f)
    return out


def closure(files: list[Path]) -> list[Path]:
    seen: list[Path] = []
    stack = list(files)
    while stack:
        f = stack.pop(0)
        if f in seen:
            continue
        seen.append(f)
        stack.extend(includes(f))
    return seen


def rel(p: Path) -> str:
    return str(p.relative_to(REF))


def main(out: Path = OUT):
    surface = {"reference": str(REF), "scripts": {}}
    for script, dropins in DROPINS.items():
        sp = REF / script
        inc = includes(sp)
        keep = [f for f in inc if any(rel(f).endswith(k) for k in KEEP_PATTERNS)]
        replace = [f for f in inc if f not in keep]
        keep_all = [f for f in closure(keep) if any(rel(f).endswith(k) for k in KEEP_PATTERNS)]
        repl_all = [f for f in closure(replace) if f not in keep_all]
        defs, structs_r, structs_k = {}, {}, {}
        for f in repl_all:
            src = f.read_text()
            for name, meths in J.functions(src).items():
                for m in meths:
                    defs.setdefault(name, []).append({k: m[k] for k in ("required", "max", "kwargs", "varkw")}
                                                     | {"file": rel(f), "line": m["line"]})
            for name, fields in J.structs(src).items():
                structs_r[name] = {"fields": fields, "file": rel(f)}
        for f in keep_all:
            for name, fields in J.structs(f.read_text()).items():
                structs_k[name] = {"fields": fields, "file": rel(f)}
        struct_names = set(structs_r) | set(structs_k)
        full_defs = {}
        for f in repl_all:
            for name, meths in J.functions(f.read_text()).items():
                full_defs.setdefault(name, []).extend(meths)
        names = set(defs)
        calls = []
        for f in [sp] + [k for k in keep_all if k.name == "plotting.jl"]:
            for c in J.calls(f.read_text(), names):
                calls.append(c | {"file": rel(f)})
        called = sorted({c["fn"] for c in calls})
        returns = {fn: J.return_kind(fn, full_defs, struct_names) for fn in called}
        reads = [r | {"file": script} for r in J.field_reads(sp.read_text(), set(called))]
        plot = next((k for k in keep_all if k.name == "plotting.jl"), None)
        plot_reads = J.typed_param_reads(plot.read_text(), "SolvedModel") if plot else []
        surface["scripts"][script] = {
            "includes": [rel(f) for f in inc], "keep": [rel(f) for f in keep], "replace": [rel(f) for f in replace],
            "dropins": dropins, "defs": defs, "calls": calls, "returns": returns, "field_reads": reads,
            "plotting_solvedmodel_reads": plot_reads, "structs_replaced": structs_r, "structs_kept": structs_k,
        }
    out.write_text(json.dumps(surface, indent=1, ensure_ascii=False, sort_keys=True) + "\n")
    for s, d in surface["scripts"].items():
        print(s, "calls", sorted({c["fn"] for c in d["calls"]}), "returns", d["returns"])


if __name__ == "__main__":
    # optional output path (default: the committed fixture tests/golden/julia_surface.json)
    main(Path(sys.argv[1]) if len(sys.argv) > 1 else OUT)
