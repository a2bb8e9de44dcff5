"""The C ABI: libsbr.so loads in the build container and exports every entry
point include/sbr.h declares; without a GPU the product path fails loudly
(no CPU fallback)."""
import ctypes

import numpy as np
import pytest

import sbr
from sbr import _lib


def test_header_declares_the_boundary():
    syms = sbr.header_symbols()
    for s in ("sbr_init", "sbr_free", "sbr_sweep_baseline", "sbr_sweep_baseline_dev", "sbr_learn_baseline",
              "sbr_solve_point_paths", "sbr_apply_early_exit"):
        assert s in syms


def test_library_exports_every_header_symbol():
    L = sbr.load()
    missing = [s for s in sbr.header_symbols() if not hasattr(L, s)]
    assert not missing


def test_default_opts_are_the_reference_defaults():
    o = _lib.default_opts()
    assert o.ode_reltol == np.finfo(np.float64).eps == o.ode_abstol  # learning.jl:43
    assert o.ode_maxiters == 1_000_000
    assert o.bisect_max_iters == 100  # solver.jl:309
    assert o.early_exit_nan_run == 5  # 1_baseline.jl:147,221


def test_status_bits_are_distinct():
    vals = list(sbr.STATUS.values())
    assert len(vals) == len(set(vals))
    assert all(v & (v - 1) == 0 for v in vals)


def test_early_exit_post_pass_matches_oracle(oracle):
    """sbr_apply_early_exit is host code in libsbr: same result as the oracle's rule."""
    rng = np.random.default_rng(1)
    nb, nu = 7, 60
    st = np.where(rng.random((nb, nu)) < 0.6, sbr.STATUS["SBR_RUN"] | sbr.STATUS["SBR_CONVERGED"],
                  sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"]).astype(np.uint32)
    st[:, 40:] = sbr.STATUS["SBR_NO_RUN_HR_BELOW_U"]
    base = dict(xi=rng.random((nb, nu)), aw_max=rng.random((nb, nu)), tol=rng.random((nb, nu)), status=st)
    o = oracle.apply_early_exit(base, 5)
    arrs = {k: np.ascontiguousarray(v.copy()) for k, v in base.items()}
    P = ctypes.c_void_p
    soa = _lib.ResultSoA(arrs["xi"].ctypes.data_as(P), None, None, arrs["aw_max"].ctypes.data_as(P),
                         arrs["tol"].ctypes.data_as(P), arrs["status"].ctypes.data_as(P), None)
    sbr.load().sbr_apply_early_exit(nb, nu, 5, ctypes.byref(soa))
    for k in ("xi", "aw_max", "tol", "status"):
        a, b = arrs[k], o[k]
        assert np.all((a == b) | (np.isnan(a) & np.isnan(b))), k


def test_no_gpu_means_loud_failure():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(sbr.SBRNativeError):
        sbr.Engine(0)


def test_social_entry_points_validate_arguments():
    """ArgumentError mirrors for the social sweep are raised before any device work
    (no GPU needed to reach them: a null context is rejected first)."""
    import ctypes
    L = sbr.load()
    soa = sbr._lib.ResultSoA()
    rc = L.sbr_sweep_social(None, None, None, 1e-4, None, 1, 1, 0.5, 0.5, 0.5, None, 1000, 1e-4, 10, None,
                            ctypes.byref(soa), None, None)
    assert rc == sbr._lib.SBR_EARG


def test_kernel_code_provenance():
    """bench.py folds PMC counters into its roofline line only for the machine code they
    were collected on: the per-kernel code sha read from libsbr.so's gfx950 code object."""
    from sbr import provenance

    shas = {k: provenance.kernel_code_sha(k) for k in ("equilibrium_kernel<768, false>",
                                                       "equilibrium_hetero_kernel<8, 256>", "hazard_kernel",
                                                       "learn_logistic_kernel")}
    assert all(s is not None and len(s) == 16 for s in shas.values()), shas
    assert len(set(shas.values())) == len(shas)
    assert provenance.kernel_code_sha("no_such_kernel") is None
    assert provenance.kernel_base("void sbr::equilibrium_kernel<768, false>(sbr::LearnBufs)") == "equilibrium_kernel"
