"""The explicit-pdf knots-in equilibrium (sbr_equilibrium_on_knots_pdf, the social drop-in's
HR / get_AW source) on the CPU: the oracle's restatement with pdf = βG(1 − G) is the
symbolic-pdf path (solver.jl:153-185 on learning.jl:161-173's pdf).
GPU parity: tests/test_gpu_social.py::test_social_point_engine_hr_and_aw_paths,
tests/test_gpu_knots.py::test_knots_pdf_matches_oracle."""
import numpy as np


def test_oracle_pdf_path_equals_symbolic(oracle):
    beta, eta, u, p, kappa, lam = 0.8, 12.5, 0.4, 0.9, 0.6, 0.1
    t, G, _ = oracle.learn_logistic(beta, eta)
    a = oracle.equilibrium_paths(t, G, beta, eta, eta, u, p, kappa, lam)
    b = oracle.equilibrium_paths_pdf(t, G, (beta * G) * (1.0 - G), eta, eta, u, p, kappa, lam)
    for k, v in a.items():
        assert np.array_equal(np.asarray(v), np.asarray(b[k]), equal_nan=True), k
    # the hazard is a ratio: a scaled pdf gives the same HR; another shape does not
    c = oracle.equilibrium_paths_pdf(t, G, 2.0 * ((beta * G) * (1.0 - G)), eta, eta, u, p, kappa, lam)
    assert np.array_equal(c["hr_tau"], a["hr_tau"]) and np.allclose(c["hr"], a["hr"], rtol=1e-12)
    d = oracle.equilibrium_paths_pdf(t, G, ((beta * G) * (1.0 - G)) * G, eta, eta, u, p, kappa, lam)
    assert np.array_equal(d["hr_tau"], a["hr_tau"]) and not np.allclose(d["hr"], a["hr"])

