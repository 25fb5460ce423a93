"""Deterministic fp32 transcendentals (csrc/lgs_detmath.h) shared by the HIP env step and
the CPU oracle: accuracy against double-precision numpy.  The HIP side computes the same
bits (tests/test_gpu_parity.py compares the whole step bitwise)."""
import ctypes as C

import numpy as np
import pytest


@pytest.fixture(scope="module")
def dm(oracle_lib):
    oracle_lib.orc_detmath.restype = C.c_float
    oracle_lib.orc_detmath.argtypes = [C.c_int, C.c_float, C.c_float]
    return oracle_lib.orc_detmath


def ulp_err(got, want):
    got = np.asarray(got, np.float64)
    want = np.asarray(want, np.float64)
    ulp = np.spacing(np.abs(want).astype(np.float32)).astype(np.float64)
    ulp = np.maximum(ulp, np.finfo(np.float32).tiny)
    return np.abs(got - want) / ulp


def run(fn, which, a, b=None):
    b = np.zeros_like(a) if b is None else b
    return np.array([fn(which, float(x), float(y)) for x, y in zip(a, b)], np.float32)


@pytest.mark.parametrize("which,f,lo,hi,maxulp", [
    (0, np.sin, -40.0, 40.0, 2.0), (1, np.cos, -40.0, 40.0, 2.0),
    (2, np.exp, -86.0, 10.0, 2.0), (4, np.arcsin, -1.0, 1.0, 3.0)])
def test_unary_accuracy(dm, which, f, lo, hi, maxulp):
    x = np.random.default_rng(which).uniform(lo, hi, 20000).astype(np.float32)
    x = np.concatenate([x, np.array([0.0, -0.0, lo, hi, 0.5, -0.5, 1e-6, np.pi / 4, np.pi / 2, np.pi], np.float32)])
    x = x[(x >= lo) & (x <= hi)]
    got = run(dm, which, x)
    err = ulp_err(got, f(x.astype(np.float64)))
    if which in (0, 1):  # absolute error near the zeros of sin/cos (argument reduction)
        err = np.minimum(err, np.abs(got - f(x.astype(np.float64))) / np.finfo(np.float32).eps)
    assert err.max() <= maxulp, (which, float(err.max()), x[np.argmax(err)])


def test_exp_underflow_and_range(dm):
    assert dm(2, -100.0, 0.0) == 0.0
    assert dm(2, 0.0, 0.0) == 1.0
    assert np.isfinite(dm(2, 88.0, 0.0))


def test_atan2_accuracy_and_signs(dm):
    rng = np.random.default_rng(7)
    y = rng.normal(0, 3, 20000).astype(np.float32)
    x = rng.normal(0, 3, 20000).astype(np.float32)
    got = run(dm, 3, y, x)
    err = ulp_err(got, np.arctan2(y.astype(np.float64), x.astype(np.float64)))
    assert err.max() <= 3.0, float(err.max())
    for yy, xx in ((0.0, 1.0), (-0.0, 1.0), (0.0, -1.0), (-0.0, -1.0), (1.0, 0.0), (-1.0, 0.0), (0.0, 0.0),
                   (0.0, -0.0), (-0.0, -0.0), (5.0, 1e-30), (1e-30, 5.0)):
        want = np.arctan2(np.float32(yy), np.float32(xx))
        got = dm(3, yy, xx)
        assert abs(got - want) <= 4e-7 * max(1.0, abs(want)) and np.signbit(got) == np.signbit(want), (yy, xx, got, want)
