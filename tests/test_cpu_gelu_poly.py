"""The bf16 network's GELU (az_net_kernels.h gelu_poly): log2 erfc(a / sqrt2) as a P5(a) on
a = min(|v|, 5.5), GELU(v) = max(v, 0) - |v| exp2(a P5(a) - 1).  Its coefficients are read from
the kernel header and evaluated in f32 step by step (the kernel's fma order) over a dense grid:
the absolute error against the f64 erf form stays under 2.9e-7 (the A&S 7.1.26 form it
replaced: 3.3e-7)."""
import os
import re

import numpy as np
from scipy.special import erf

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "master_doko_reinforcement_learning_amd", "csrc", "az_net_kernels.h")


def _coefficients():
    src = open(HDR).read()
    body = src[src.index("float gelu_poly(float v)"):]
    body = body[:body.index("}")]
    first = float(re.search(r"float q = (-?[0-9.e+-]+)f;", body).group(1))
    rest = [float(x) for x in re.findall(r"q = fmaf\(q, a, (-?[0-9.e+-]+)f\);", body)]
    return np.array([first] + rest, dtype=np.float32)   # highest degree first


def _fma32(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


def test_gelu_poly_error_bound():
    c = _coefficients()
    assert len(c) == 6
    v = np.concatenate([np.linspace(-12.0, 12.0, 2_000_001), np.linspace(-1e4, 1e4, 2_000_001),
                        -np.logspace(0.5, 4, 10001), np.logspace(0.5, 4, 10001)]).astype(np.float32)
    a = np.minimum(np.abs(v), np.float32(5.5))
    q = np.full_like(a, c[0])
    for k in c[1:]:
        q = _fma32(q, a, np.full_like(a, k))
    e = np.exp2(_fma32(q, a, np.full_like(a, -1.0))).astype(np.float32)
    e = np.where(np.abs(v) > np.float32(5.5), np.float32(0.0), e).astype(np.float32)
    g = _fma32(-np.abs(v), e, np.maximum(v, np.float32(0.0)))
    ref = 0.5 * v.astype(np.float64) * (1.0 + erf(v.astype(np.float64) / np.sqrt(2.0)))
    assert np.abs(g - ref).max() < 2.9e-7
