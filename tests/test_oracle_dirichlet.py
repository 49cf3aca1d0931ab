"""The oracle's rand_distr 0.5.1 restatement (oracle/rand_distr05.hpp) against the moments of
the distributions it samples.  The reference holds no vector for these draws (the crate is a
crates.io dependency, Cargo.lock:1948-1949), so the draws themselves are PARITY UNPINNED; these
checks pin the algorithms' distributions, and tests/native/dirichlet_check.cpp pins the device
code to this restatement draw for draw."""
import ctypes

import numpy as np
import pytest

import oracle_lib as ol


def _rng(seed):
    return ol.rng_seed(seed)


def _z(x, mean, var, n):
    """z-score of a sample mean against the exact mean (standard error from the exact variance)."""
    return abs(float(np.mean(x)) - mean) / np.sqrt(var / n)


@pytest.mark.parametrize("alpha", [0.05, 0.1, 0.5, 0.8, 1.0, 2.5])
def test_dirichlet_moments(alpha):
    """Dirichlet([alpha; 39]) (async_mcts.rs:111): 10^6 draws; every component has mean 1/39 and
    variance alpha (a0 - alpha) / (a0^2 (a0 + 1)), a0 = 39 alpha; each draw sums to 1.  alpha <= 0.1
    takes the crate's FromBeta stick-breaking construction (components may underflow to 0 in f32)."""
    n, k = 1_000_000, 39
    out = np.zeros(n * k, dtype=np.float32)
    rng = _rng(1234 + int(alpha * 10))
    assert ol.lib().or_dirichlet(ctypes.c_float(alpha), k, n, rng, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))) == 1
    x = out.reshape(n, k).astype(np.float64)
    assert np.all(x > 0) if alpha > 0.1 else np.all(x >= 0)
    assert np.allclose(x.sum(axis=1), 1.0, atol=1e-5)
    a0 = k * alpha
    mean, var = 1.0 / k, alpha * (a0 - alpha) / (a0 * a0 * (a0 + 1.0))
    for j in (0, 13, 38):
        assert _z(x[:, j], mean, var, n) < 5.0
        assert abs(np.var(x[:, j]) / var - 1.0) < 0.02
    # components are identically distributed: the pooled mean of every column
    assert _z(x.ravel(), mean, var, n * k) < 5.0 * np.sqrt(k)


@pytest.mark.parametrize("shape", [0.3, 0.8, 1.0, 1.5, 4.0])
def test_gamma_moments(shape):
    """Gamma(shape, 1): mean = variance = shape (Marsaglia-Tsang, the small-shape boost, Exp)."""
    n = 1_000_000
    out = np.zeros(n, dtype=np.float32)
    ol.lib().or_gamma(ctypes.c_float(shape), n, _rng(77), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    x = out.astype(np.float64)
    assert _z(x, shape, shape, n) < 5.0
    assert abs(np.var(x) / shape - 1.0) < 0.02


def test_ziggurat_normal_and_exp():
    """StandardNormal (mean 0, var 1, symmetric tails past R = 3.654) and Exp1 (mean 1, var 1)."""
    n = 2_000_000
    z = np.zeros(n)
    ol.lib().or_normal_f64(n, _rng(5), z.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    assert _z(z, 0.0, 1.0, n) < 5.0 and abs(np.var(z) - 1.0) < 0.01
    tail = np.mean(np.abs(z) > 3.6541528853610088)
    assert abs(tail - 2.58e-4) < 5 * np.sqrt(2.58e-4 / n)   # P(|Z| > R) = 2.58e-4
    e = np.zeros(n)
    ol.lib().or_exp1_f64(n, _rng(6), e.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    assert np.all(e >= 0) and _z(e, 1.0, 1.0, n) < 5.0 and abs(np.var(e) - 1.0) < 0.02
    assert abs(np.mean(e > 7.69711747013104972) - np.exp(-7.69711747013104972)) < 5 * np.sqrt(4.5e-4 / n)


def test_ziggurat_tables_shape():
    """The regenerated tables: x decreasing from v/f(R) to 0, f = pdf(x) increasing to 1, and
    the crate's first layers (rand_distr src/ziggurat_tables.rs opens with these values)."""
    t = np.zeros(1030)
    ol.lib().or_ziggurat_tables(t.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    nx, nf, ex, ef = t[:257], t[257:514], t[514:771], t[771:1028]
    for x, f in ((nx, nf), (ex, ef)):
        assert np.all(np.diff(x) < 0) and x[-1] == 0.0 and np.all(np.diff(f) > 0) and f[-1] == 1.0
    assert "%.18f" % nx[0] == "3.910757959537090045" and "%.18f" % nx[2] == "3.449278298560964462"
    assert "%.18f" % nf[0] == "0.000477467764586655" and "%.18f" % t[1028] == "3.654152885361008796"


@pytest.mark.parametrize("a,b", [(0.1, 3.8), (0.05, 0.05), (0.5, 0.5), (3.0, 0.7), (2.5, 4.0), (1.5, 1.2)])
def test_beta_moments(a, b):
    """Beta(a, b) (Cheng's BC for min(a, b) <= 1, BB otherwise; the parameter switch both ways):
    mean a / (a + b), variance a b / ((a + b)^2 (a + b + 1)) over 10^6 draws."""
    n = 1_000_000
    out = np.zeros(n, dtype=np.float32)
    ol.lib().or_beta(ctypes.c_float(a), ctypes.c_float(b), n, _rng(31), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    x = out.astype(np.float64)
    assert np.all((x >= 0) & (x <= 1))
    s = a + b
    mean, var = a / s, a * b / (s * s * (s + 1.0))
    assert _z(x, mean, var, n) < 5.0
    assert abs(np.var(x) / var - 1.0) < 0.02
