"""The Julia binding (replication-social-bank-runs_amd/julia/SBREngine.jl + SBRDropIn.jl)
cannot run here (no Julia in the image), so its contract with include/sbr.h is checked
statically: the `struct Opts` / `struct ResultSoA` mirrors have the C structs' field
offsets and sizes (a C program compiled against sbr.h prints offsetof / sizeof), the
ctypes mirror agrees, every ccall'd symbol is declared in sbr.h and exported by libsbr,
and every ccall passes as many arguments as the C prototype takes."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
JL = REPO / "replication-social-bank-runs_amd" / "julia"
HEADER = REPO / "include" / "sbr.h"

# Julia isbits field types → (size, alignment) of the C layout Julia uses for them
JL_TYPES = {"Float64": (8, 8), "Int64": (8, 8), "Int32": (4, 4), "UInt32": (4, 4)}


def jl_struct_fields(name):
    src = (JL / "SBREngine.jl").read_text()
    m = re.search(r"^struct %s\b.*?\n(.*?)^end" % name, src, re.S | re.M)
    assert m, name
    fields = []
    for line in m.group(1).splitlines():
        line = line.split("#")[0].strip()
        if not line:
            continue
        f, t = line.split("::")
        t = t.strip()
        fields.append((f.strip(), (8, 8) if t.startswith("Ptr{") else JL_TYPES[t]))
    return fields


def jl_layout(fields):
    off, out, align = 0, {}, 1
    for f, (sz, al) in fields:
        off = (off + al - 1) // al * al
        out[f] = off
        off += sz
        align = max(align, al)
    return out, (off + align - 1) // align * align


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    d = tmp_path_factory.mktemp("layout")
    prog = d / "layout.c"
    fields = {"sbr_opts": [f for f, _ in jl_struct_fields("Opts")],
              "sbr_result_soa": [f for f, _ in jl_struct_fields("ResultSoA")]}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for st, fs in fields.items():
        lines.append(f'printf("{st} sizeof %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0; }")
    prog.write_text("\n".join(lines))
    exe = d / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(prog)], check=True)
    out = {}
    for line in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        st, f, v = line.split()
        out[(st, f)] = int(v)
    return out


@pytest.mark.parametrize("jl_name, c_name", [("Opts", "sbr_opts"), ("ResultSoA", "sbr_result_soa")])
def test_julia_struct_layout_matches_header(c_layout, jl_name, c_name):
    offs, size = jl_layout(jl_struct_fields(jl_name))
    assert size == c_layout[(c_name, "sizeof")]
    for f, o in offs.items():
        assert o == c_layout[(c_name, f)], (jl_name, f)


def test_ctypes_mirror_matches_header(c_layout):
    from sbr import _lib

    for cls, c_name in ((_lib.Opts, "sbr_opts"), (_lib.ResultSoA, "sbr_result_soa")):
        assert ctypes.sizeof(cls) == c_layout[(c_name, "sizeof")]
        for f, _ in cls._fields_:
            assert getattr(cls, f).offset == c_layout[(c_name, f)], (c_name, f)


def _prototypes():
    src = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(?:int|void|const char\*|sbr_ctx\*)\s+(sbr_\w+)\s*\(([^)]*)\)\s*;", src):
        args = [a for a in m.group(2).split(",") if a.strip() and a.strip() != "void"]
        protos[m.group(1)] = len(args)
    return protos


def _ccalls():
    calls = []
    for f in JL.glob("*.jl"):
        src = f.read_text()
        for m in re.finditer(r"ccall\(\(:(\w+), libsbr\),\s*\w+(?:\{\w+\})?,\s*\(", src):
            # the argument-type tuple: balance parentheses from the match end
            i, depth = m.end(), 1
            while depth:
                depth += {"(": 1, ")": -1}.get(src[i], 0)
                i += 1
            types = src[m.end():i - 1]
            n = len([t for t in re.split(r",(?![^{]*\})", types) if t.strip()])
            calls.append((f.name, m.group(1), n))
    return calls


def test_julia_ccalls_match_prototypes():
    protos = _prototypes()
    calls = _ccalls()
    assert len(calls) >= 10
    for fname, sym, n in calls:
        assert sym in protos, (fname, sym)
        assert n == protos[sym], (fname, sym, n, protos[sym])


def test_ccalled_symbols_are_exported():
    from sbr import _lib

    L = _lib.load()
    for _, sym, _ in _ccalls():
        assert hasattr(L, sym), sym


def test_dropin_defines_the_reference_call_surface():
    """SBRDropIn.jl defines what scripts/1_baseline.jl and plotting.jl call (learning.jl /
    solver.jl names) with the reference's SolvedModel / LearningResults fields."""
    src = (JL / "SBRDropIn.jl").read_text()
    for fn in ("solve_learning", "solve_equilibrium_baseline", "get_AW_functions!", "get_AW", "hazard_rate",
               "compute_pdf_symbolic_baseline"):
        assert re.search(r"^function %s\(" % re.escape(fn), src, re.M), fn
    for st, fields in (("LearningResults", ("params", "learning_cdf", "learning_pdf", "grid", "solve_time",
                                            "ode_solution")),
                       ("SolvedModel", ("ξ", "τ_bar_IN_UNC", "τ_bar_OUT_UNC", "HR", "bankrun", "τ_IN", "τ_OUT",
                                        "model_params", "learning_results", "converged", "solve_time", "tolerance",
                                        "aw"))):
        body = re.search(r"^struct %s\b(.*?)^end" % st, src, re.S | re.M).group(1)
        declared = re.findall(r"^\s+(\w+)::", body, re.M)
        assert tuple(declared[:len(fields)]) == fields, (st, declared)


# --------------------------------------------------------------------------------------
# The extension drop-ins: every script switches by include.  The reference
# surface per script (calls, arities, returns, fields read) comes from the reference's own
# files via tools/extract_julia_surface.py → tests/golden/julia_surface.json.
import json  # noqa: E402
import sys  # noqa: E402

sys.path.insert(0, str(Path(__file__).resolve().parent))
import jl_surface as JS  # noqa: E402

SURFACE = json.loads((REPO / "tests" / "golden" / "julia_surface.json").read_text())["scripts"]


def _dropin_defs(files):
    defs, structs, full = {}, {}, {}
    for f in files:
        src = (JL / f).read_text()
        for name, meths in JS.functions(src).items():
            full.setdefault(name, []).extend(meths)
        structs.update(JS.structs(src))
    return full, structs


@pytest.mark.parametrize("script", sorted(SURFACE))
def test_dropins_define_every_called_function_with_reference_arity(script):
    s = SURFACE[script]
    defs, _ = _dropin_defs(s["dropins"])
    assert s["calls"], script
    for c in s["calls"]:
        meths = defs.get(c["fn"])
        assert meths, f"{script}: {c['fn']} (called at {c['file']}:{c['line']}) is not defined by {s['dropins']}"
        ok = any(m["required"] <= c["npos"] <= (m["max"] if m["max"] is not None else 1 << 30)
                 and (m["varkw"] or set(c["kwargs"]) <= set(m["kwargs"])) for m in meths)
        assert ok, (script, c, [(m["required"], m["max"], m["kwargs"]) for m in meths])
        # and with the reference's own signature (positional range and keywords)
        for r in s["defs"][c["fn"]]:
            if r["required"] <= c["npos"] <= (r["max"] if r["max"] is not None else 1 << 30):
                assert any(m["required"] == r["required"] and m["max"] == r["max"]
                           and set(r["kwargs"]) <= set(m["kwargs"]) for m in meths), (script, c["fn"], r)


@pytest.mark.parametrize("script", sorted(SURFACE))
def test_dropins_return_the_reference_result_types(script):
    s = SURFACE[script]
    defs, structs = _dropin_defs(s["dropins"])
    names = set(structs) | set(s["structs_kept"]) | set(s["structs_replaced"])
    for fn, kind in s["returns"].items():
        if kind is None:  # an interpolant (hazard_rate)
            continue
        mine = JS.return_kind(fn, defs, names)
        assert mine == kind, (script, fn, mine, kind)


@pytest.mark.parametrize("script", sorted(SURFACE))
def test_dropins_provide_every_field_the_scripts_and_plotting_read(script):
    s = SURFACE[script]
    defs, structs = _dropin_defs(s["dropins"])
    # structs the replaced files defined: the drop-ins define them with the reference's fields, in order
    for name, st in s["structs_replaced"].items():
        assert name in structs, (script, name, st["file"])
        assert structs[name][:len(st["fields"])] == st["fields"], (script, name, structs[name], st["fields"])

    def fields_of(kind):
        if "namedtuple" in kind:
            return kind["namedtuple"]
        n = kind["struct"]
        return structs[n] if n in structs else s["structs_kept"][n]["fields"]

    for r in s["field_reads"]:
        kind = s["returns"][r["fn"]]
        assert kind is not None, r
        assert r["field"] in fields_of(kind), (script, r)
    for f in s["plotting_solvedmodel_reads"]:
        assert f in structs["SolvedModel"], (script, f)


def test_surface_fixture_matches_reference_when_present(tmp_path):
    """The fixture is what tools/extract_julia_surface.py reads from /root/reference today
    (skipped where the reference is absent, e.g. on the GPU box).  The extractor writes to a
    temporary file: the committed fixture is compared, never rewritten."""
    if not Path("/root/reference/scripts").is_dir():
        pytest.skip("reference not present")
    import subprocess as sp

    fresh = tmp_path / "julia_surface.json"
    out = sp.run([sys.executable, str(REPO / "tools" / "extract_julia_surface.py"), str(fresh)], capture_output=True,
                 text=True)
    assert out.returncode == 0, out.stderr
    assert fresh.read_text() == (REPO / "tests" / "golden" / "julia_surface.json").read_text()
