"""ctypes binding of libsbr.so (include/sbr.h).

The product path has no CPU fallback: if the shared library or a GPU is
missing, the calls raise ``SBRNativeError``.
"""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent  # replication-social-bank-runs_amd/
REPO_ROOT = PKG_ROOT.parent
LIB_PATH = Path(os.environ["SBR_LIB"]) if os.environ.get("SBR_LIB") else PKG_ROOT / "lib" / "libsbr.so"
HEADER = REPO_ROOT / "include" / "sbr.h"
STATUS_HEADER = REPO_ROOT / "include" / "sbr_status.h"

_D = ctypes.c_double
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_P = ctypes.c_void_p

SBR_OK, SBR_EARG, SBR_EDEVICE, SBR_ENOMEM = 0, -1, -2, -3
SBR_FLAG_EXHAUSTIVE = 0x1
SBR_FLAG_READY_SWEEP = 0x2
SBR_FLAG_RCCL_GATHER = 0x4
SBR_FLAG_XI_GUESS = 0x8
SBR_FLAG_DIAG_STOP_AFTER_BUFFER = 0x100
SBR_FLAG_DIAG_STOP_AFTER_BISECT = 0x200
SBR_FLAG_DIAG_COUNT_AW_BLOCKS = 0x400
SBR_FLAG_DIAG_SOCIAL_PROF = 0x800


class SBRNativeError(RuntimeError):
    """The native engine is unavailable or returned an error."""


class ArgumentError(ValueError):
    """Mirror of Julia's ArgumentError raised by the reference's constructors."""


class Opts(ctypes.Structure):
    _fields_ = [
        ("ode_reltol", _D),
        ("ode_abstol", _D),
        ("ode_maxiters", _I64),
        ("bisect_max_iters", _I32),
        ("early_exit_nan_run", _I32),
        ("knot_capacity", _I32),
        ("hetero_max_iters", _I32),
        ("flags", _I32),
        ("pad", _I32),  # social sweep knot capacity per buffer (0 = 98304)
        ("xi_guess", _D),  # compute_ξ's first iterate (NaN: the midpoint); knots-in calls only
    ]


class ResultSoA(ctypes.Structure):
    _fields_ = [
        ("xi", _P),
        ("tau_in_unc", _P),
        ("tau_out_unc", _P),
        ("aw_max", _P),
        ("tol", _P),
        ("status", _P),
        ("iters", _P),
    ]


def _parse_status_bits() -> dict[str, int]:
    bits = {}
    for m in re.finditer(r"#define\s+(SBR_\w+)\s+(0x[0-9a-fA-F]+)u", STATUS_HEADER.read_text()):
        bits[m.group(1)] = int(m.group(2), 16)
    return bits


STATUS = _parse_status_bits()
globals().update(STATUS)

_SIGS = {
    "sbr_default_opts": (None, [_P]),
    "sbr_init": (ctypes.c_int, [ctypes.c_int, _P]),
    "sbr_init_multi": (ctypes.c_int, [ctypes.c_int, _P, _P]),
    "sbr_multi_size": (ctypes.c_int, [_P]),
    "sbr_multi_child": (_P, [_P, ctypes.c_int]),
    "sbr_free": (ctypes.c_int, [_P]),
    "sbr_last_error": (ctypes.c_char_p, [_P]),
    "sbr_sweep_baseline": (ctypes.c_int, [_P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _P]),
    "sbr_sweep_baseline_dev": (ctypes.c_int, [_P, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _P]),
    "sbr_sweep_baseline_batch_dev": (ctypes.c_int, [_P, _P, _I64, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P,
                                                    _P]),
    "sbr_batch_wait": (ctypes.c_int, [_P, _P, _I64]),
    "sbr_batch_reserve": (ctypes.c_int, [_P, _I64, _I64, _P]),
    "sbr_set_batch_workspace": (ctypes.c_int, [_P, _I64]),
    "sbr_learn_baseline": (ctypes.c_int, [_P, _P, _P, _P, _D, _I64, _I32, _P, _P, _P, _I64, _P, _P]),
    "sbr_solve_point_paths": (ctypes.c_int, [_P, _D, _D, _D, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "sbr_equilibrium_on_knots": (ctypes.c_int, [_P, _P, _P, _I64, _D, _D, _D, _P, _I64, _D, _D, _D, _P, _P, _P, _P,
                                                _P, _P, _P, _I64, _P]),
    "sbr_equilibrium_on_knots_pdf": (ctypes.c_int, [_P, _P, _P, _P, _I64, _D, _D, _P, _I64, _D, _D, _D, _P, _P, _P,
                                                    _P, _P, _P, _P, _I64, _P]),
    "sbr_hetero_equilibrium_on_knots": (ctypes.c_int, [_P, _I32, _P, _P, _I64, _P, _P, _D, _D, _P, _I64, _D, _D, _D,
                                                       _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "sbr_apply_early_exit": (None, [_I64, _I64, _I32, _P]),
    "sbr_selftest_detmath": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, _P, _P, _P]),
    "sbr_timing_enable": (ctypes.c_int, [_P, ctypes.c_int]),
    "sbr_last_schedule": (ctypes.c_int, [_P, _P]),
    "sbr_host_phases": (ctypes.c_int, [_P, _P]),
    "sbr_chunk_timeline": (ctypes.c_int, [_P, _P, _P, _P]),
    "sbr_timing_read": (ctypes.c_int, [_P, _P, _P, _P, _P]),
    "sbr_learn_stats": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, _P]),
    "sbr_hetero_learn_stats": (ctypes.c_int, [_P, _I64, _P, _P, _P, _P, _P]),
    "sbr_selftest_fastpow": (ctypes.c_int, [_P, _P, _P, ctypes.c_int, _P]),
    "sbr_device_info": (ctypes.c_int, [_P, _P, _P, _P]),
    "sbr_sweep_hetero": (ctypes.c_int, [_P, _I32, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _P, _P, _P]),
    "sbr_sweep_hetero_dev": (ctypes.c_int, [_P, _P, _I32, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _P, _P,
                                            _P]),
    "sbr_sweep_hetero_batch_dev": (ctypes.c_int, [_P, _P, _I64, _I32, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D,
                                                  _D, _P, _P, _P, _P]),
    "sbr_sweep_social": (ctypes.c_int, [_P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _I32, _D, _I32, _P, _P, _P,
                                        _P]),
    "sbr_sweep_social_dev": (ctypes.c_int, [_P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _P, _I32, _D, _I32, _P,
                                            _P, _P, _P]),
    "sbr_set_social_workspace": (ctypes.c_int, [_P, _I64]),
    "sbr_social_prof_read": (ctypes.c_int, [_P, _P]),
    "sbr_social_overflow_stats": (ctypes.c_int, [_P, _P, _P]),
    "sbr_social_point_paths": (ctypes.c_int, [_P, _D, _D, _D, _D, _D, _D, _D, _P, ctypes.c_int32, _D,
                                              ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "sbr_learn_hetero": (ctypes.c_int, [_P, _I32, _P, _P, _P, _D, _I64, _P, _P, _P, _I64, _P, _P]),
    "sbr_hetero_point_paths": (ctypes.c_int, [_P, ctypes.c_int32, _P, _P, _D, _D, _D, _D, _D, _D, _D, _P, _P, _P,
                                              _P, _P, _P, _P, _P, _P, _I64, _P]),
    "sbr_interest_point_paths": (ctypes.c_int, [_P, _D, _D, _D, _D, _D, _D, _D, _D, _D, _D, _P, _P, _P, _P, _P, _P,
                                                _P, _I64, _P, _P]),
    "sbr_sweep_interest": (ctypes.c_int, [_P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _D, _D, _P, _P, _P]),
    "sbr_sweep_interest_dev": (ctypes.c_int, [_P, _P, _P, _P, _P, _D, _P, _I64, _I64, _D, _D, _D, _D, _D, _P, _P,
                                              _P]),
}

_lib: ctypes.CDLL | None = None


def header_symbols() -> list[str]:
    """Every function declared in include/sbr.h."""
    src = HEADER.read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(sbr_\w+)\s*\(", src, re.M)))


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise SBRNativeError(
            f"{LIB_PATH} is missing: build it with `make -C {PKG_ROOT}` (or __graft_entry__.build()); "
            "there is no CPU fallback")
    L = ctypes.CDLL(str(LIB_PATH))
    for name, (res, args) in _SIGS.items():
        # an older libsbr.so loaded for an A/B (SBR_LIB) may lack a newer entry point: calling it
        # then raises AttributeError; tests/test_capi.py asserts the built library exports them all
        fn = getattr(L, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def default_opts(**kw) -> Opts:
    o = Opts()
    load().sbr_default_opts(ctypes.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def check(rc: int, ctx=None, what: str = "sbr call"):
    if rc == SBR_OK:
        return
    msg = ""
    if ctx is not None:
        m = load().sbr_last_error(ctx)
        msg = m.decode() if m else ""
    if rc == SBR_EARG:
        raise ArgumentError(f"{what}: {msg}")
    raise SBRNativeError(f"{what} failed ({rc}): {msg}")
