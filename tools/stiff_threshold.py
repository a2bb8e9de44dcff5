#!/usr/bin/env python3
"""The AutoSwitch stiffness test |eigen_est·dt / 3.5068| > 9/10 (OrdinaryDiffEqCore is_stiff,
alg_stability_size(::Tsit5) = 3.5068) as one compare: x ↦ fl(x / 3.5068) is monotone, so
fl(x / 3.5068) > 0.9 ⟺ x ≥ T for the least double T passing the test.  Prints T (hex),
used by sbr_device.h AutoSwitch::STIFF_THRESHOLD; tests/test_oracle_golden.py re-checks it."""
import struct


def threshold(c: float = 3.5068, tol: float = 0.9) -> float:
    f = lambda x: abs(x / c) > tol  # noqa: E731  (IEEE division, correctly rounded)
    lo, hi = 0, struct.unpack("<Q", struct.pack("<d", 4 * c * tol))[0]
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if f(struct.unpack("<d", struct.pack("<Q", mid))[0]):
            hi = mid
        else:
            lo = mid
    return struct.unpack("<d", struct.pack("<Q", hi))[0]


if __name__ == "__main__":
    print(threshold().hex())
