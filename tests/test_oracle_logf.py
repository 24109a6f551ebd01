"""The precise tile cull's logf (rasterizer_impl.cu:151: keep a (tile, Gaussian) pair when max_contrib_power <=
logf(co.w / (1/255)), CUDA's logf, <= 1 ulp).  The oracle and the kernels evaluate the correctly rounded logf
(gs_crlogf: one IEEE-double operation sequence shared with gs_common.h), the closest stand-in for CUDA's.

* exhaustive: gs_crlogf equals logl rounded once to float on every float in [2^-20, 256) -- a superset of the cull's
  arguments o * 255, o in (2^-24, 1];
* independent of libm: at 80 decimal digits (Python's decimal), gs_crlogf is the correctly rounded value on the two
  inputs whose exact logarithm lies within 3e-16 of a float midpoint (where the double evaluation alone misrounds) and
  on a seeded sample of 4000 cull arguments;
* the census of round 5's float polynomial is recorded in profiles/r06_logf_census.json (tools/logf_census.py).
"""
from decimal import Decimal, getcontext

import numpy as np


def _cr_decimal(x: float) -> np.float32:
    """The float nearest to ln(x), ties to even, from an 80-digit logarithm."""
    getcontext().prec = 80
    exact = Decimal(float(x)).ln()
    f = np.float32(float(exact))             # within one float ulp of the exact value
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
    dist = [abs(Decimal(float(c)) - exact) for c in cands]
    best = min(range(3), key=lambda i: dist[i])
    return cands[best]


def test_crlogf_exhaustive_against_logl(oracle):
    n_bad, bad = oracle.crlogf_check(0x35800000, 0x43800000)     # [2^-20, 256)
    assert n_bad == 0, [float(b).hex() for b in bad]


def test_crlogf_near_midpoints_and_sample_against_decimal(oracle):
    xs = [float.fromhex("0x1.827a74p-7"), float.fromhex("0x1.2f1fd6p+3"), 1.0, 255.0, 1.0 / 255.0 * 255.0]
    rng = np.random.default_rng(6)
    o = rng.uniform(1.0 / 255.0, 1.0, 4000).astype(np.float32)
    xs += list((o / np.float32(1.0 / 255.0)).astype(np.float32))
    for x in xs:
        got = np.float32(oracle.gs_crlogf(x))
        assert got == _cr_decimal(x), (float(x).hex(), float(got).hex(), float(_cr_decimal(x)).hex())


def test_cull_threshold_is_logf_of_the_quotient(oracle):
    """cull_log_threshold(o) = gs_crlogf(o / (1/255)) with the float division first, as rasterizer_impl.cu:151."""
    o = np.array([1.0, 0.5, 1.0 / 255.0, 0.003, 0.99, 2.0 ** -24], np.float32)
    q = (o / np.float32(1.0 / 255.0)).astype(np.float32)
    want = np.array([oracle.gs_crlogf(float(v)) for v in q], np.float32)
    np.testing.assert_array_equal(oracle.cull_log_threshold(o), want)
