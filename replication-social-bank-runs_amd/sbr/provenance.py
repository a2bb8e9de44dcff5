"""Provenance of measured kernel data (bench.py, tools/pmc_summary.py).

PMC counters are collected in separate rocprofv3 runs; bench.py folds them into its
roofline line (``traffic``, ``frac_executed``) only when they were collected on the
same kernel machine code.  A kernel is identified by the sha256 of its gfx950 code
bytes inside libsbr.so (every instantiation of the kernel template, read from the
clang offload bundle's code object), so rebuilding an unrelated kernel does not
invalidate the counters of the equilibrium kernel, and any change to its own code does.
"""
from __future__ import annotations

import hashlib
import struct
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent
REPO_ROOT = PKG_ROOT.parent
_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_base(kernel: str) -> str:
    """'void sbr::equilibrium_kernel<768, false>(...)' -> 'equilibrium_kernel'."""
    k = kernel.replace("void ", "").replace("sbr::", "")
    return k.split("<")[0].split("(")[0].strip()


def _code_objects(blob: bytes):
    """gfx950 ELF code objects of every clang offload bundle in a host binary."""
    pos = blob.find(_BUNDLE_MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", blob, pos + 24)
        off = pos + 32
        for _ in range(n):
            o, size, tl = struct.unpack_from("<QQQ", blob, off)
            triple = blob[off + 24: off + 24 + tl].decode(errors="replace")
            off += 24 + tl
            if "gfx950" in triple and size:
                yield blob[pos + o: pos + o + size]
        pos = blob.find(_BUNDLE_MAGIC, pos + 24)


def _symbols(elf: bytes):
    """(name, bytes) of every STT_FUNC symbol with a size in an ELF64 code object."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    for s in secs:
        if s[1] != 2:  # SHT_SYMTAB
            continue
        strtab = secs[s[6]]
        for j in range(s[5] // 24):
            name_off, info, _, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s[4] + j * 24)
            if (info & 0xF) != 2 or size == 0 or shndx >= shnum:  # STT_FUNC
                continue
            end = elf.index(b"\0", strtab[4] + name_off)
            name = elf[strtab[4] + name_off: end].decode(errors="replace")
            sec = secs[shndx]
            fo = sec[4] + (value - sec[3])
            yield name, elf[fo: fo + size]


def kernel_code_sha(kernel: str, lib: Path | str | None = None) -> str | None:
    """sha256 (16 hex) over the code bytes of every instantiation of `kernel`'s template in
    libsbr.so (symbols sorted by mangled name), or None if none is found."""
    from . import _lib

    base = kernel_base(kernel)
    tag = f"{len(base)}{base}"  # Itanium mangling of the unqualified name
    blob = Path(lib or _lib.LIB_PATH).read_bytes()
    found = sorted((n, b) for co in _code_objects(blob) for n, b in _symbols(co) if tag in n)
    if not found:
        return None
    h = hashlib.sha256()
    for n, b in found:
        h.update(n.encode())
        h.update(b)
    return h.hexdigest()[:16]
