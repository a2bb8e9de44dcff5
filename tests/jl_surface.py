"""A small static reader of Julia source (no Julia in the image): top-level function
definitions with their positional / keyword arguments, struct fields, the kind of value a
function returns (a struct it constructs or a NamedTuple's keys), call sites with their
arity, and field reads on variables.  Used by tools/extract_julia_surface.py (on the
reference's files → tests/golden/julia_surface.json) and tests/test_julia_shim.py (on the
drop-ins).  Regex + bracket matching: good for the code style of both sides, not a parser."""
from __future__ import annotations

import re

IDENT = r"[A-Za-z_\u0080-￿][A-Za-z0-9_!\u0080-￿]*"


def strip_comments(src: str) -> str:
    src = re.sub(r"#=.*?=#", lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    # docstrings """…""" (keep line count)
    src = re.sub(r'"""(.*?)"""', lambda m: "\n" * m.group(0).count("\n"), src, flags=re.S)
    out = []
    for line in src.split("\n"):
        # drop `# …` outside string literals
        q, cut = False, len(line)
        for i, ch in enumerate(line):
            if ch == '"' and (i == 0 or line[i - 1] != "\\"):
                q = not q
            elif ch == "#" and not q:
                cut = i
                break
        out.append(line[:cut])
    return "\n".join(out)


def _match_paren(s: str, i: int) -> int:
    """s[i] == '(' → index just past its matching ')'."""
    depth, q = 0, False
    for j in range(i, len(s)):
        ch = s[j]
        if ch == '"' and s[j - 1] != "\\":
            q = not q
        if q:
            continue
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
            if depth == 0:
                return j + 1
    raise ValueError("unbalanced")


def split_top(s: str, sep: str = ",") -> list[str]:
    parts, depth, cur, q = [], 0, "", False
    for j, ch in enumerate(s):
        if ch == '"' and (j == 0 or s[j - 1] != "\\"):
            q = not q
        if not q:
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            elif ch == sep and depth == 0:
                parts.append(cur)
                cur = ""
                continue
        cur += ch
    if cur.strip():
        parts.append(cur)
    return [p.strip() for p in parts if p.strip()]


def parse_args(inner: str) -> dict:
    """Argument list text → {required, max, kwargs, varkw}."""
    semi = _first_depth0(inner, ";")
    pos_s, kw_s = (inner[:semi], inner[semi + 1:]) if semi >= 0 else (inner, "")
    pos = split_top(pos_s)
    req = sum(1 for a in pos if "=" not in a.replace("==", "") and not a.endswith("..."))
    varpos = any(a.endswith("...") for a in pos)
    kws, varkw = [], False
    for a in split_top(kw_s):
        if a.endswith("..."):
            varkw = True
            continue
        kws.append(re.split(r"[:=]", a, 1)[0].strip())
    return {"required": req, "max": None if varpos else len(pos), "kwargs": kws, "varkw": varkw}


def _first_depth0(s: str, target: str) -> int:
    depth = 0
    for j, ch in enumerate(s):
        if ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == target and depth == 0:
            return j
    return -1


def _block_end(src: str, start: int) -> int:
    """Index just past the `end` closing the block opened at `start` (a line with
    function/struct/…); counts block keywords line by line."""
    opens = re.compile(r"\b(function|if|for|while|let|begin|struct|mutable struct|try|do|quote|module)\b")
    depth = 0
    pos = start
    for line in src[start:].split("\n"):
        code = re.sub(r'"[^"]*"', '""', line)
        # bracketed text holds no blocks: x[end], comprehensions / generators `(… for …)`
        prev = None
        while prev != code:
            prev = code
            code = re.sub(r"\([^()]*\)|\[[^\[\]]*\]", "", code)
        # one-line `if … end` etc. count both
        depth += len(opens.findall(code))
        depth -= len(re.findall(r"\bend\b", code))
        # a short-form definition `f(x) = …` never opens a block
        pos += len(line) + 1
        if depth <= 0:
            return pos
    return len(src)


def functions(src: str) -> dict[str, list[dict]]:
    """Top-level (column 0) function definitions: name → list of methods
    {required, max, kwargs, varkw, line, body}."""
    src = strip_comments(src)
    out: dict[str, list[dict]] = {}
    for m in re.finditer(r"^function\s+(%s)\s*\(" % IDENT, src, re.M):
        i = m.end() - 1
        j = _match_paren(src, i)
        sig = parse_args(src[i + 1:j - 1])
        end = _block_end(src, m.start())
        sig.update(line=src[:m.start()].count("\n") + 1, body=src[j:end])
        out.setdefault(m.group(1), []).append(sig)
    for m in re.finditer(r"^(%s)\s*\(" % IDENT, src, re.M):  # short form f(args) = expr
        i = m.end() - 1
        j = _match_paren(src, i)
        rest = src[j:j + 40]
        if not re.match(r"\s*(::\s*\w+\s*)?=(?!=)", rest):
            continue
        sig = parse_args(src[i + 1:j - 1])
        eol = src.find("\n\n", j)
        sig.update(line=src[:m.start()].count("\n") + 1, body=src[j:eol if eol > 0 else len(src)])
        out.setdefault(m.group(1), []).append(sig)
    return out


def structs(src: str) -> dict[str, list[str]]:
    """struct name → field names in order (inner constructors skipped)."""
    src = strip_comments(src)
    out = {}
    for m in re.finditer(r"^(?:mutable\s+)?struct\s+(%s)\b[^\n]*\n" % IDENT, src, re.M):
        end = _block_end(src, m.start())
        body = src[m.end():end]
        fields, depth = [], 0
        for line in body.split("\n"):
            s = line.strip()
            if depth == 0 and re.match(r"^(function\b|%s\s*\(.*\)\s*=)" % IDENT, s):
                depth += 1
                continue
            if depth > 0:
                depth += len(re.findall(r"\b(function|if|for|while|let|begin|try)\b", s))
                depth -= len(re.findall(r"\bend\b", s))
                continue
            fm = re.match(r"^(%s)\s*(::.*)?$" % IDENT, s)
            if fm and fm.group(1) != "end":
                fields.append(fm.group(1))
        out[m.group(1)] = fields
    return out


def namedtuple_keys(body: str) -> list[str] | None:
    """Keys of the last NamedTuple literal `(k1 = …, k2 = …)` in a function body."""
    found = None
    for m in re.finditer(r"\(\s*(%s)\s*=(?!=)" % IDENT, body):
        try:
            j = _match_paren(body, m.start())
        except ValueError:
            continue
        parts = split_top(body[m.start() + 1:j - 1])
        keys = []
        for p in parts:
            km = re.match(r"^(%s)\s*=(?!=)" % IDENT, p)
            if not km:
                keys = None
                break
            keys.append(km.group(1))
        if keys and len(keys) >= 2:
            found = keys
    return found


def return_kind(name: str, defs: dict[str, list[dict]], struct_names: set[str], _seen=None) -> dict | None:
    """What function `name` returns: {"struct": S} if its body returns a constructed struct
    (directly, through a variable, or through another function of `defs`), {"namedtuple":
    keys} for a NamedTuple literal.  First method whose body decides it."""
    _seen = set() if _seen is None else _seen
    if name in _seen or name not in defs:
        return None
    _seen.add(name)
    for meth in defs[name]:
        body = meth["body"]
        for m in re.finditer(r"\breturn\s+(%s)\s*(\(|$|\n)" % IDENT, body, re.M):
            tok = m.group(1)
            if tok in struct_names:
                return {"struct": tok}
            if tok in defs and tok != name:
                r = return_kind(tok, defs, struct_names, _seen)
                if r:
                    return r
            # return var: follow `var = X(` assignments
            for a in re.finditer(r"\b%s\s*=\s*(%s)\s*\(" % (re.escape(tok), IDENT), body):
                f = a.group(1)
                if f in struct_names:
                    return {"struct": f}
                r = return_kind(f, defs, struct_names, _seen)
                if r:
                    return r
        keys = namedtuple_keys(body)
        if keys:
            return {"namedtuple": keys}
        for c in re.finditer(r"\b(%s)\s*\(" % IDENT, body):
            f = c.group(1)
            if f in defs and f != name and ("aw" in body or "return" in body):
                r = return_kind(f, defs, struct_names, _seen)
                if r and "namedtuple" in r:
                    return r
    return None


def calls(src: str, names: set[str]) -> list[dict]:
    """Call sites `f(args…)` of the given function names: {fn, npos, kwargs, line}."""
    src = strip_comments(src)
    out = []
    for m in re.finditer(r"(?<![\w.!])(%s)\s*\(" % IDENT, src):
        fn = m.group(1)
        if fn not in names:
            continue
        line_start = src.rfind("\n", 0, m.start()) + 1
        if re.match(r"\s*function\s", src[line_start:m.start()]):
            continue
        j = _match_paren(src, m.end() - 1)
        inner = src[m.end():j - 1]
        semi = _first_depth0(inner, ";")
        pos_s, kw_s = (inner[:semi], inner[semi + 1:]) if semi >= 0 else (inner, "")
        pos, kws = [], []
        for a in split_top(pos_s):
            km = re.match(r"^(%s)\s*=(?!=)" % IDENT, a)
            (kws.append(km.group(1)) if km else pos.append(a))
        kws += [re.split(r"=", a, 1)[0].strip() for a in split_top(kw_s)]
        out.append({"fn": fn, "npos": len(pos), "kwargs": kws, "line": src[:m.start()].count("\n") + 1})
    return out


def field_reads(src: str, producers: set[str]) -> list[dict]:
    """Variables assigned from a producer call (`v = f(…)`) and the fields read on them
    (`v.field`, `(; a, b) = v`): {var, fn, field, line}."""
    src = strip_comments(src)
    bind = {}
    for m in re.finditer(r"^\s*(%s)\s*=\s*(%s)\s*\(" % (IDENT, IDENT), src, re.M):
        if m.group(2) in producers:
            bind[m.group(1)] = m.group(2)
    out = []
    for var, fn in bind.items():
        for m in re.finditer(r"(?<![\w.])%s\.(%s)" % (re.escape(var), IDENT), src):
            out.append({"var": var, "fn": fn, "field": m.group(1), "line": src[:m.start()].count("\n") + 1})
        for m in re.finditer(r"\(;\s*([^)]*)\)\s*=\s*%s\b(?!\.)" % re.escape(var), src):
            for f in split_top(m.group(1)):
                out.append({"var": var, "fn": fn, "field": f, "line": src[:m.start()].count("\n") + 1})
    return out


def typed_param_reads(src: str, type_name: str) -> list[str]:
    """Fields read on a function parameter annotated `::type_name` (plotting.jl's
    `result::SolvedModel`), incl. `(; a, b) = param`."""
    src = strip_comments(src)
    fields = []
    for m in re.finditer(r"^function\s+%s\s*\(" % IDENT, src, re.M):
        i = m.end() - 1
        j = _match_paren(src, i)
        pm = re.search(r"(%s)::%s\b" % (IDENT, re.escape(type_name)), src[i:j])
        if not pm:
            continue
        p = pm.group(1)
        body = src[j:_block_end(src, m.start())]
        fields += re.findall(r"(?<![\w.])%s\.(%s)" % (re.escape(p), IDENT), body)
        for d in re.finditer(r"\(;\s*([^)]*)\)\s*=\s*%s\b(?!\.)" % re.escape(p), body):
            fields += split_top(d.group(1))
    return sorted(set(fields))
