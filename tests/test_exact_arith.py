"""Exactness of the arithmetic shortcuts the HIP kernels take (CPU only).

The kernels must reproduce the reference's IEEE-754 float32 results bit for
bit (north_star), so every replacement of an IEEE division is proven here
over its whole input domain, in exact rational arithmetic.
"""
from fractions import Fraction as Fr

import numpy as np


def rn32(x):
    """Round a Fraction to the nearest float32, ties to even (exactly)."""
    f = np.float32(float(x))
    cands = [f, np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))]

    def key(c):
        bits = int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0])
        return (abs(Fr(float(c)) - x), bits & 1)
    return np.float32(min(cands, key=key))


def fma32(a, b, c):
    return rn32(Fr(float(a)) * Fr(float(b)) + Fr(float(c)))


def test_u8_unit_exact():
    # prk_device.h u8_unit: (float)k / 255.0f == fma(fma(-255, q0, k), c, q0),
    # q0 = k * c, c = RN(1/255) = 0x1.010102p-8, for every byte value k
    # (the texel channel conversion of projekt.cpp:2029-2032 and 441-446).
    c = np.float32(float.fromhex("0x1.010102p-8"))
    assert c == rn32(Fr(1, 255))
    for k in range(256):
        kf = np.float32(k)
        q0 = rn32(Fr(k) * Fr(float(c)))
        rem = fma32(np.float32(-255.0), q0, kf)
        got = fma32(rem, c, q0)
        assert got == rn32(Fr(k, 255)), k


def test_focal_power_of_two_exact():
    # prk_device.h div_focal: d / F == d * (1/F) when F = 2^k (single rounding
    # of the same exact value); spot-check normal, tiny and huge d.
    rng = np.random.default_rng(0)
    ds = np.concatenate([rng.standard_normal(2000).astype(np.float32),
                         np.float32([1e-38, -3e-39, 7e37, 0.0, -0.0, 4.0])])
    for F in [1.0, 2.0, 0.5, 8.0, 2.0 ** -20, 2.0 ** 40]:
        F32 = np.float32(F)
        inv = np.float32(1.0) / F32
        with np.errstate(over="ignore", under="ignore"):
            a = ds / F32
            b = ds * inv
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), F
