"""hf_div / hf_sqrt (core/common.hpp), the division and square root every
GPU step kernel uses, against IEEE division / square root (numpy, the host
build): bit for bit over operands spanning 10^-300 .. 10^300, the physical
ranges of the solver, and the zero / infinite / NaN special cases (kept by
v_div_fixup).  The GPU == CPU bitwise tests of the step kernels rest on it."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(x):
    return np.asarray(x, dtype=np.float64).view(np.uint64)


def test_hf_div_sqrt_bitwise_equal_ieee(gpu):
    rng = np.random.default_rng(7)
    n = 1 << 20
    ea = rng.uniform(-300, 300, n)
    eb = rng.uniform(-300, 300, n)
    keep = np.abs(ea - eb) < 300   # quotients inside the normal range
    a = (rng.uniform(1, 10, n) * 10.0 ** ea * rng.choice([-1, 1], n))[keep]
    b = (rng.uniform(1, 10, n) * 10.0 ** eb * rng.choice([-1, 1], n))[keep]
    # physical operands of the step kernels (densities, pressures, residuals ...)
    phys = rng.uniform(1e-6, 1e7, 200000)
    a = np.concatenate([a, phys, rng.uniform(-1, 1, 200000)])
    b = np.concatenate([b, phys[::-1], rng.uniform(1e-3, 2, 200000)])
    q, s = gpu.native().div_probe(a, b)
    np.testing.assert_array_equal(_bits(q), _bits(a / b))
    with np.errstate(invalid="ignore"):
        ref_s = np.sqrt(np.abs(a))
    q2, s2 = gpu.native().div_probe(np.abs(a), b)
    np.testing.assert_array_equal(_bits(s2), _bits(ref_s))


def test_hf_div_special_operands(gpu):
    vals = np.array([0.0, -0.0, 1.0, -2.5, np.inf, -np.inf, 1e-300, 3e300])
    a = np.repeat(vals, len(vals))
    b = np.tile(vals, len(vals))
    q, s = gpu.native().div_probe(a, b)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        ref = a / b
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(q), nan)
    np.testing.assert_array_equal(_bits(q[~nan]), _bits(ref[~nan]))
    # sqrt: zero (either sign) and +inf pass through, a steady cell's zero residual
    z = np.array([0.0, -0.0, np.inf, 4.0, 2.0])
    _, sz = gpu.native().div_probe(z, np.ones_like(z))
    np.testing.assert_array_equal(_bits(sz), _bits(np.sqrt(z)))
